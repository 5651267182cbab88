#!/bin/bash
# tests + smoke + bench (tools/gpu_round.sh), then the in-kernel phase stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_round.sh || exit $?
timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps.log 2>&1
rc=$?; tail -6 gpurun_out/stamps.log; exit $rc
