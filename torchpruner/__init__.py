"""Import-compatible alias of :mod:`torchpruner_amd` under the reference's package name, so
code written against TorchPruner (``from torchpruner.attributions import ...``,
``from torchpruner.pruner import Pruner``) runs unchanged on the MI355X engine."""
from torchpruner_amd import *  # noqa: F401,F403
from torchpruner_amd import __all__, __version__  # noqa: F401
