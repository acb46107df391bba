#!/bin/bash
# round 6, call d: the fp16x2 GRU forward's accuracy and time with the fourth product a2 b2 and / or activations
# scaled by 2^4 before their split (A/B builds libmarlsat_{a2b2,asc4,both}.so), then the train-cycle margins
# over four seeds on the variants
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=marl-sat_amd/marlsat/lib
for lib in libmarlsat libmarlsat_a2b2 libmarlsat_asc4 libmarlsat_both; do
  MARLSAT_LIB=$PWD/$L/$lib.so timeout -k 10 120 python -u profiles/gru_h2_accuracy.py 70000 \
      >> gpurun_out/r06d_gru_accuracy.log 2>&1 || { echo "accuracy $lib failed"; tail -5 gpurun_out/r06d_gru_accuracy.log; exit 1; }
done
grep -E "lib|h2r|x3r|plain" gpurun_out/r06d_gru_accuracy.log | cut -c1-160
for i in 1 2; do
  for lib in libmarlsat libmarlsat_a2b2 libmarlsat_asc4 libmarlsat_both; do
    echo "== $lib $i" >> gpurun_out/r06d_gru_time.log
    MARLSAT_LIB=$PWD/$L/$lib.so timeout -k 10 120 python -u profiles/gru_r_bench.py >> gpurun_out/r06d_gru_time.log 2>&1 \
        || { echo "time $lib failed"; exit 1; }
  done
done
grep -E "==|h2r" gpurun_out/r06d_gru_time.log | cut -c1-200
for lib in libmarlsat_a2b2 libmarlsat_both; do
  MARLSAT_LIB=$PWD/$L/$lib.so timeout -k 10 400 python -u profiles/parity_switch_probe.py --seeds 4,5,6,7 default \
      > gpurun_out/r06d_probe_$lib.log 2>&1 || { echo "probe $lib failed"; tail -5 gpurun_out/r06d_probe_$lib.log; exit 1; }
  echo "probe $lib:"; grep -o "margins [^ ]* .*step [0-9]\|grad worst ratio [0-9.e-]* ([^)]*)" gpurun_out/r06d_probe_$lib.log | paste - - | sed 's/V100 C430 A10 H128 L16 mode0//'
done
