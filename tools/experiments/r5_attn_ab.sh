#!/bin/bash
# prev (libvtd_prev.so) vs new attention: tests, attn_bench at C2 (B 256, N 196) and C3 (B 32,
# N 1600) interleaved, then C2 B=256 and C3 B=32 forwards interleaved (3 rounds each).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-attn_ab}; mkdir -p $O
P=$R/vision_transformer_detector_amd/libvtd_prev.so
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attention or batch_parity" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for shp in "c2:--B 256 --N 196" "c3:--B 32 --N 1600"; do
    lab=${shp%%:*}; args=${shp#*:}
    VTD_LIB_PATH=$P timeout -k 10 60 python tools/attn_bench.py --reps 30 $args > $O/attn_${lab}_p$r.log 2>&1 || exit 1
    timeout -k 10 60 python tools/attn_bench.py --reps 30 $args > $O/attn_${lab}_n$r.log 2>&1 || exit 1
    echo "attn $lab r$r prev $(grep -o '"us": [0-9.]*' $O/attn_${lab}_p$r.log) new $(grep -o '"us": [0-9.]*' $O/attn_${lab}_n$r.log)"
  done
done
for r in 1 2 3; do
  for cfg in "c2:--batch 256" "c3:--preset vit_b16_640 --batch 32"; do
    lab=${cfg%%:*}; args=${cfg#*:}
    VTD_LIB_PATH=$P timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 20 $args > $O/p_${lab}_$r.log 2>&1 || { tail -5 $O/p_${lab}_$r.log; exit 1; }
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity-mode --steps 20 $args > $O/n_${lab}_$r.log 2>&1 || { tail -5 $O/n_${lab}_$r.log; exit 1; }
    echo "fwd $lab r$r prev $(tail -1 $O/p_${lab}_$r.log | grep -o '"value": [0-9.]*') new $(tail -1 $O/n_${lab}_$r.log | grep -o '"value": [0-9.]*')"
  done
done
