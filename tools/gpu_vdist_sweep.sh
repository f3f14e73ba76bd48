#!/bin/bash
# vdist rehearsal under several engine environments (VCONFIGS: ";"-separated
# VAR=value lists, "-" = defaults); args: N K S...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra CFG <<< "${VCONFIGS:--}"
n=0
for cfg in "${CFG[@]}"; do
  n=$((n + 1))
  envs=()
  [ "$cfg" != - ] && read -ra envs <<< "$cfg"
  echo "== $cfg"
  timeout -k 10 300 env "${envs[@]}" python -u tools/vdist_rehearsal.py "$@" > gpurun_out/vsw_$n.log 2>&1 || { tail -20 gpurun_out/vsw_$n.log; exit 1; }
  cut -c1-330 gpurun_out/vsw_$n.log
done
