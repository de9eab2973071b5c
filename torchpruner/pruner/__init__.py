from torchpruner_amd.pruner import *  # noqa: F401,F403
from torchpruner_amd.pruner import __all__  # noqa: F401
