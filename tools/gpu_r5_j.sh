#!/bin/bash
# Round 5: where the early coarse backward (--coarse-stream) pays: 1024 / 2048 rays,
# graph-replayed and eager, with and without, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 1024 2048; do
  for g in "--graph" ""; do
    for i in 1 2; do
      for cs in "" "--coarse-stream"; do
        tag=b${B}${g:+g}${cs:+_cs}_$i
        timeout -k 10 300 python bench.py --batch $B $g --steps 100 --warmup 10 --no-cpu-baseline $cs > gpurun_out/r5j_$tag.json 2> gpurun_out/r5j_$tag.err || { tail -n 20 gpurun_out/r5j_$tag.err; exit 3; }
        python -c "import json;d=json.load(open('gpurun_out/r5j_$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
      done
    done
  done
done
