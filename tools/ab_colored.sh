#!/bin/bash
# Colored-noise fold A/B: GPU tests of the augment chain, then the headline's augment stage
# timing with the fold (default) and without (HBK_AUG_NO_COLORED_FOLD=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 300 python -u -m pytest tests/test_augment.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
