set -e
mkdir -p gpurun_out/r04z/gaps8
export TMPDIR=/tmp
run() { # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04z/gaps8/$tag -o k -- python3 tools/run_overhead.py --reps 1 > gpurun_out/r04z/gaps8/$tag.log 2>&1
  f=$(ls gpurun_out/r04z/gaps8/$tag/*kernel_trace.csv | head -1)
  python3 tools/gap_stats.py $f 20 > gpurun_out/r04z/gaps8/$tag.txt
}
run fixed ICP_X=1
env timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04z/gaps8/w8 -o k -- python3 tools/shard_probe.py --worlds 8 --steps 30 --warmup 3 > gpurun_out/r04z/gaps8/w8.log 2>&1
python3 tools/gap_stats.py $(ls gpurun_out/r04z/gaps8/w8/*kernel_trace.csv | head -1) 20 > gpurun_out/r04z/gaps8/w8.txt
