set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/sprof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --sharded > $O/sprof.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/spmc_fetch -o run --output-format csv -- python3 bench.py --steps 40 --warmup 8 --no-cpu-baseline --sharded > $O/spmc_fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/spmc_write -o run --output-format csv -- python3 bench.py --steps 40 --warmup 8 --no-cpu-baseline --sharded > $O/spmc_write.log 2>&1
timeout -k 10 60 python tools/profile_summary.py --tag r01_sharded --prof $O/sprof --fetch $O/spmc_fetch --write $O/spmc_write --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline --sharded (PMC: separate --pmc FETCH_SIZE / WRITE_SIZE passes, --steps 40 --warmup 8)" > $O/ssum.log 2>&1
mkdir -p $O/profiles_out && cp profiles/r01_sharded_* $O/profiles_out/
grep -o '"ms_per_step": [0-9.]*' $O/sprof.log
