#!/bin/bash
# Experiment build of the engine with extra defines: tools/build_exp.sh <tag> "-DFOO=1 ..."
# -> build_exp/libsa_<tag>.so (load it with SA_HIP_LIB=...). Development only.
set -e
tag=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
src=${SRC_DIR:-$root/sequence-alignment-gpu_amd/csrc}  # SRC_DIR: build other sources (e.g. a git worktree's)
out=/tmp/sa_build_exp/$tag
mkdir -p "$out"
# GEN_ENV="SA_GEN_BAND_PF_STEP=14 ..." regenerates the fill steps with those generator settings into a
# copy of the sources
if [ -n "$GEN_ENV" ]; then
  rm -rf "$out/src" && cp -r "$src" "$out/src"
  env $GEN_ENV SA_GEN_FILL_OUT="$out/src/sa_fill_steps.inc" python3 "$root/tools/gen_fill_asm.py" >/dev/null
  src=$out/src
fi
flags="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$root/include -I$src -DSA_EXPERIMENT=1 $*"
# EXP_ONLY="fill_r1 ..." recompiles only those units and takes the others from the product build
pids=()
for f in sa_engine sa_walk sa_batch fill_r1 fill_r1a fill_r2 fill_r4 fill_r8 fill_r16 fill_r32; do
  if [ -n "$EXP_ONLY" ] && [[ " $EXP_ONLY " != *" $f "* ]]; then
    cp $root/sequence-alignment-gpu_amd/build/$f.o $out/$f.o
  else
    /opt/rocm/bin/hipcc $flags -c $src/$f.hip -o $out/$f.o & pids+=($!)
  fi
done
for p in "${pids[@]}"; do wait $p; done
mkdir -p $root/build_exp
cp $root/sequence-alignment-gpu_amd/build/build_id.o $out/build_id.o
/opt/rocm/bin/hipcc $flags -shared $out/*.o -L/opt/rocm/lib -ldl -o $root/build_exp/libsa_$tag.so
rm -f $root/build_exp/libsa_$tag.so.[0-9]*
echo built build_exp/libsa_$tag.so
