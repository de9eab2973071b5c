#!/bin/bash
# Parity check: run the reference's OWN unit tests (torchpruner/tests, 26 tests: the attribution
# goldens and the pruner NaN-trick / optimizer cases) unchanged against this package, which
# answers `import torchpruner`. The test files are copied to a scratch dir (never into the repo)
# so that `torchpruner` resolves to our alias package, not the reference's.
#   bash scripts/run_reference_tests.sh [/root/reference]
set -euo pipefail
REF=${1:-/root/reference}
REPO=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
cp "$REF"/torchpruner/tests/test_attributions.py "$REF"/torchpruner/tests/test_pruner.py "$TMP"/
cd "$TMP"
PYTHONPATH="$REPO" python -m pytest -q -p no:cacheprovider .
