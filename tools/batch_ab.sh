# A/B runs at C4 (60 steps) and the W = 8 shard
set -e
bash tools/env_ab.sh r04z/errpair ICP_ERR_PAIR "1 0 1 0"
bash tools/env_ab.sh r04z/trb2 ICP_TR_BATCH "1 2 1 2"
bash tools/env_ab.sh r04z/xcd ICP_GRID_XCD "1 2 1 2"
bash tools/env_ab.sh r04z/fused ICP_FUSED_STEPS "0 1 2 3 0 1 2 3"
