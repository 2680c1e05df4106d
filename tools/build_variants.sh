#!/bin/bash
# Builds libexacto_hip.so variants that differ only in ntt.hip compile flags, for A/B runs of
# tools/ntt_bench.py / bench.py with EXACTO_HIP_LIB=build/variants/<name>.so.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
make -C $R/exacto_amd/csrc -s
OUT=$R/build/variants; mkdir -p $OUT
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC"
build() {  # name, flags...
  local name=$1; shift
  $H "$@" -c $R/exacto_amd/csrc/ntt.hip -o $OUT/ntt_$name.o
  $H --offload-arch=gfx950 -shared -fPIC -o $OUT/$name.so $R/build/obj/context.o $R/build/obj/kernels.o \
    $R/build/obj/keygen.o $R/build/obj/plain.o $R/build/obj/ks32.o $OUT/ntt_$name.o -ldl
}
# a variant whose generated rounds differ (gen_ntt_asm.py env switches): ntt.hip is compiled from a
# copy next to the regenerated ntt_asm.inc (quoted includes search the file's own directory first)
build_gen() {  # name, env assignment
  local name=$1; shift
  local D=$OUT/src_$name; mkdir -p $D
  cp $R/exacto_amd/csrc/ntt.hip $D/
  env "$@" python3 -c "import sys; sys.path.insert(0, '$R/tools'); import gen_ntt_asm as G; G.OUT = '$D/ntt_asm.inc'; G.main()" > /dev/null
  $H -I $R/exacto_amd/csrc -c $D/ntt.hip -o $OUT/ntt_$name.o
  $H --offload-arch=gfx950 -shared -fPIC -o $OUT/$name.so $R/build/obj/context.o $R/build/obj/kernels.o \
    $R/build/obj/keygen.o $R/build/obj/plain.o $R/build/obj/ks32.o $OUT/ntt_$name.o -ldl
}
for v in "$@"; do
  case $v in
    base) build base ;;
    as0) build as0 -DEXACTO_TW_AS=0 ;;
    as1) build as1 -DEXACTO_TW_AS=1 ;;
    as1_w4) build as1_w4 -DEXACTO_TW_AS=1 -DEXACTO_NTT_WAVES=4 ;;
    as4_w4) build as4_w4 -DEXACTO_NTT_WAVES=4 ;;
    nopre) build nopre -DEXACTO_NTT_PRELOAD=0 ;;
    nopre_w5) build nopre_w5 -DEXACTO_NTT_PRELOAD=0 -DEXACTO_NTT_WAVES=5 ;;
    nopre_w6) build nopre_w6 -DEXACTO_NTT_PRELOAD=0 -DEXACTO_NTT_WAVES=6 ;;
    w5) build w5 -DEXACTO_NTT_WAVES=5 ;;
    ilp) build ilp -mllvm -amdgpu-sched-strategy=max-ilp ;;
    ilp_w3) build ilp_w3 -mllvm -amdgpu-sched-strategy=max-ilp -DEXACTO_NTT_WAVES=3 ;;
    nomulasm) build nomulasm -DEXACTO_MUL_ASM=0 ;;
    ld1st0) build ld1st0 -DEXACTO_BUF_ST=0 ;;
    ld0st1) build ld0st1 -DEXACTO_BUF_LD=0 ;;
    ld0st0) build ld0st0 -DEXACTO_BUF_LD=0 -DEXACTO_BUF_ST=0 ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
done
