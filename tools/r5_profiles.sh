#!/bin/bash
# round-5 profiles of every single-GPU config at the in-tree library: rocprofv3 kernel trace + stats, then
# FETCH_SIZE and WRITE_SIZE in passes of their own (tools/profile_round.sh); outputs gpurun_out/p5<cfg>_*
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for c in ${CONFIGS:-c1 c2 c3 c4}; do
  PROF_ARGS="--config $c --steps 16 --warmup 4 --prof-steps 0 --cpu-sample 0 --no-check --decode-steps 4 --drain-steps 0 --h2d-steps 0" \
    T_PROF=240 tools/profile_round.sh || exit 1
  for x in trace fetch write; do rm -rf gpurun_out/p5${c}_$x; mv gpurun_out/prof_$x gpurun_out/p5${c}_$x; done
  for x in trace fetch write; do mv gpurun_out/prof_$x.log gpurun_out/p5${c}_$x.log; done
  cp gpurun_out/prof_md5.txt gpurun_out/p5${c}_md5.txt
done
exit 0
