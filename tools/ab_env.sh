#!/bin/bash
# A/B of environment knobs on a bench script: tools/ab_env.sh <script.py> "name:ENV=V ..." ...
# (two rounds; prints the script's JSON lines per variant)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
script=$1; shift
for round in 1 2; do
for spec in "$@"; do
  IFS=: read -r name envs <<< "$spec"
  env $envs timeout -k 10 300 python "$script" > gpurun_out/abe_$(basename $script .py)_$name.log 2>&1 || exit $?
  echo "== $name (round $round)"
  grep '^{' gpurun_out/abe_$(basename $script .py)_$name.log | cut -c1-200
done
done
