# A/B of the streaming kernels' load batches at C4 (60 steps) and the W = 8 shard
set -e
bash tools/env_ab.sh r04z/trb2 ICP_TR_BATCH "1 2 1 2"
