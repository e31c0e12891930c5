#!/bin/bash
# GPU box: sampler A/B below 65,536 sockets, then configs[4]'s eps = 0.42 point resumed to the
# reference's 200 frame errors.
set -u
bash scripts/r03l.sh || exit $?
ENS_POINTS=0.42 ENS_SECONDS=${ENS_SECONDS:-700} ENS_LIMIT=800 bash scripts/r03_ens.sh
