"""Reference package path: torchpruner.attributions.methods."""
