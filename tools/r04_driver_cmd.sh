#!/bin/bash
# Round 4: the driver's exact bench command, plain (x2) and under rocprofv3
# --kernel-trace --stats, plus the host enqueue probe -- itemises the gap
# between the kernel's rocprof average and ms_per_step.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
O=gpurun_out/r04
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_plain_$i.json 2> $O/driver_plain_$i.err || exit $?
  tail -1 $O/driver_plain_$i.json
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/steps200.json 2> $O/steps200.err || exit $?
tail -1 $O/steps200.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_prof.json 2> $O/driver_prof.err || exit $?
tail -1 $O/driver_prof.json
timeout -k 10 300 python3 tools/host_overhead.py > $O/host_overhead.txt 2>&1 || exit $?
cat $O/host_overhead.txt
find $O/prof_driver -name "*stats*" | head
