#!/bin/bash
# Minibatch A/B (tools/gpu/mbw_ab.sh, its parity subset first), then the full validation of the
# in-tree library (tools/gpu/full_check.sh: pytest -m gpu, smoke, default bench line).
bash tools/gpu/mbw_ab.sh ${1:-2} && bash tools/gpu/full_check.sh
