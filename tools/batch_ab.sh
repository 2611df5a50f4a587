# A/B runs at C4 (60 steps) and the W = 8 shard
set -e
bash tools/env_ab.sh r04z/drain ICP_GRID_DRAIN "0 1 0 1"
