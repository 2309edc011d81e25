# Tiles kernels A/B (round 5): the product build against tools/fwalt/libilqr_hip_tilesbase.so
# (the previous commit), B = 4096 × T = 100 and B = 1 × T = 1000, then the tiles tests.
set -o pipefail
for rep in 1 2; do
  for lib in "" tools/fwalt/libilqr_hip_tilesbase.so; do
    echo "== ${lib:-product}"
    ILQR_LIB=$lib timeout -k 10 120 python -u tools/ab_lib.py tools/bench_tiles.py 4096 100 2>/dev/null | grep -v '"nx": 4,' || exit 1
    ILQR_LIB=$lib timeout -k 10 120 python -u tools/ab_lib.py tools/bench_tiles.py 1 1000 2>/dev/null | grep -v '"nx": 4,' || exit 1
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tiles.py 2>&1 | tail -2
