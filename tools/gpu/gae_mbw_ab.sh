#!/bin/bash
# GAE A/B then minibatch-kernel A/B (tools/gpu/gae_ab.sh, tools/gpu/mbw_ab.sh)
bash tools/gpu/mbw_ab.sh 2 "cheetah4096 cartpole4096 lunar8192" && bash tools/gpu/gae_ab.sh
