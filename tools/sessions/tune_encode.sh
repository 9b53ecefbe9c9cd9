#!/bin/bash
# Build row-scan variants of liblac.so (here) or bench them (on the GPU box):
#   tools/sessions/tune_encode.sh build        -> tools/tune/liblac_<variant>.so
#   tools/sessions/tune_encode.sh run [args]   -> one bench line per variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
if [ "${1:-}" = build ]; then
    mkdir -p tools/tune
    rm -f tools/tune/*.so
    IFS=' '; for v in ${TUNE_VARIANTS:-base enc4 enc3 dec0}; do
        case $v in
          base) f="";;
          enc4) f="-DLAC_ENC_MINW=4";; enc3) f="-DLAC_ENC_MINW=3";;
          dec0) f="-DLAC_DEC_MINW=0";; dec3) f="-DLAC_DEC_MINW=3";; dec2) f="-DLAC_DEC_MINW=2";; decf4) f="-DLAC_DECF_MINW=4";; decf3) f="-DLAC_DECF_MINW=3";;
          u8_nt) f="-DLAC_UNROLL=8 -DLAC_NT=1";; u16_nt) f="-DLAC_UNROLL=16 -DLAC_NT=1";;
          u8_plain) f="-DLAC_UNROLL=8 -DLAC_NT=0";; u16_plain) f="-DLAC_UNROLL=16 -DLAC_NT=0";;
          u4_nt) f="-DLAC_UNROLL=4 -DLAC_NT=1";;
          imax0) f="-DLAC_Q1_IMAX=0";;
          xpf0) f="-DLAC_XPF=0";; xpf1) f="-DLAC_XPF=1 -DLAC_PIPE=0";; xpf1w2) f="-DLAC_XPF=1 -DLAC_PIPE=0 -DLAC_ENC_MINW=2";;
          dxpf) f="-DLAC_DEC_XPF=1";; dstream) f="-DLAC_DEC_STREAM_ONLY=1";; dxpfw2) f="-DLAC_DEC_XPF=1 -DLAC_DECF_MINW=2";;
          pipe1w2) f="-DLAC_XPF=1 -DLAC_PIPE=1 -DLAC_ENC_MINW=2";;
          q1u4) f="-DLAC_Q1_UNROLL=4";; q1u2) f="-DLAC_Q1_UNROLL=2";; q1u16) f="-DLAC_Q1_UNROLL=16";;
          q1nt1) f="-DLAC_Q1_NT1=1";; q1plain) f="-DLAC_Q1_NT2=0";; q1w2) f="-DLAC_Q1_MINW=2";;
          q1u4w2) f="-DLAC_Q1_UNROLL=4 -DLAC_Q1_MINW=2";; q1u4w3) f="-DLAC_Q1_UNROLL=4 -DLAC_Q1_MINW=3";;
        esac
        hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -Ilac_amd/csrc $f \
            lac_amd/csrc/lac_kernels.hip -o tools/tune/liblac_$v.so || exit 1
    done
    exit 0
fi
shift
mkdir -p gpurun_out/tune
for rep in 1 2; do
  for so in tools/tune/liblac_*.so; do
    v=$(basename "$so" .so)
    LAC_LIB="$PWD/$so" timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-baseline off "$@" \
        > "gpurun_out/tune/$v.$rep.json" 2> "gpurun_out/tune/$v.$rep.err"
    rc=$?
    [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 "gpurun_out/tune/$v.$rep.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/tune/$v.$rep.json')); r=d['roofline']; print('$v', round(d['value']/1e6,2), 'Msym/s', r['kernel'], round(r['kernel_ms_per_launch'],4), 'ms', round(r['frac'],4), 'dec', round(d['parity']['decode']['achieved_GBps'] or 0), 'GB/s', d['parity']['bit_exact_vs_oracle'], d['parity']['round_trip_all_streams'])"
  done
done
