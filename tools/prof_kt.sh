cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ktg -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5
