from torchpruner_amd.attributions import *  # noqa: F401,F403
from torchpruner_amd.attributions import __all__, _AttributionMetric  # noqa: F401
