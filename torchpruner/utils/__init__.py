from torchpruner_amd.utils import *  # noqa: F401,F403
from torchpruner_amd.utils import __all__  # noqa: F401
