#!/bin/bash
# Round-end measurements of the shipped build on one GPU box: per workload a kernel trace + FETCH/WRITE PMC
# summary (tools/gpu_profile.sh; the summaries carry the build hash) and the bench line, then the GPU suite.
#   R=r05_v2 [WORKLOADS="c3 c2 c4 c5"] bash tools/final_round.sh
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
R=${R:-rNN}
for w in ${WORKLOADS:-c3 c2 c4 c5}; do
  tag=${R}; [ "$w" != c3 ] && tag=${R}_$w
  echo "== profile $w"; date
  # the traced fold respaced (the same kernels per step; rocprofv3 crashed tracing a full 100-step C4 fold)
  st=""; [ "$w" = c2 ] && st=100; [ "$w" = c4 ] && st=20; [ "$w" = c5 ] && st=25
  STEPS=$st TAG=$tag WORKLOAD=$w bash tools/gpu_profile.sh > gpurun_out/${tag}_profile.txt 2>&1 || { tail -20 gpurun_out/${tag}_profile.txt; exit 1; }
  # the summaries come back through gpurun_out (profiles/ on the box does not); the databases stay behind
  mkdir -p gpurun_out/profiles_out && cp profiles/${tag}_* gpurun_out/profiles_out/
  rm -rf gpurun_out/prof_${tag} gpurun_out/pmc_fetch_${tag} gpurun_out/pmc_write_${tag}
  echo "== bench $w"; date
  extra=""; [ "$w" != c3 ] && extra="--steps 1 --warmup 1"
  timeout -k 10 900 python3 bench.py --workload $w $extra > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
    || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
  cat gpurun_out/${tag}_bench.json
done
