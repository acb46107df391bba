set -e
for lib in "" ab/wwabl1.so ab/wwabl2.so ab/wwabl4.so ab/wwabl3.so; do
  echo "== ${lib:-current}"
  env ${lib:+MARLSAT_LIB=$PWD/$lib} WGRAD_PATHS=1i timeout -k 10 100 python -u profiles/wgrad_w_bench.py 10 | grep -v max_err
done
