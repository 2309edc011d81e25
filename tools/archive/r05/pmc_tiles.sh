# HBM traffic of the tiles backward kernels: two PMC passes (one counter set each) over
# tools/bench_tiles.py, then tools/archive/r05/pmc_tiles.py. Each pass under its own hard limit.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/tp_fetch -o run -- python tools/bench_tiles.py > gpurun_out/tp_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/tp_write -o run -- python tools/bench_tiles.py > gpurun_out/tp_write.log 2>&1 || exit $?
python tools/archive/r05/pmc_tiles.py gpurun_out/tp_fetch gpurun_out/tp_write gpurun_out/pmc_tiles.json > gpurun_out/pmc_tiles_summary.log 2>&1
