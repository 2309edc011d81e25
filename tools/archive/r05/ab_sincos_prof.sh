# A/B of the sincos fallback's calling convention on config 5's kernels and the 2-link
# bench: libilqr_hip_prevchain.so (out-pointers into the caller's s, c), _byval.so
# (returned by value), _tmp.so (out-pointers into slow-path temporaries). The three
# libraries are built on the CPU before the call (ilqr_math.h edited per variant, `make -C
# ilqr.jl_amd/csrc ../lib/libilqr_hip.so`, copied into lib/variants/) and not kept.
# Result: profiles/r05/sincos_fallback_ab_r05.log.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out && export TMPDIR=/tmp
for i in 1 2; do
  for v in prevchain byval tmp; do
    ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abs_${v}_$i -o run --output-format csv -- python tools/ab_lib.py tools/bench_rbd.py --lin fd --no-cpu --steps 50 --warmup 50 > gpurun_out/abs_${v}_$i.log 2>&1 || exit $?
    ILQR_LIB=ilqr.jl_amd/lib/variants/libilqr_hip_$v.so timeout -k 10 200 python tools/ab_lib.py tools/bench_twolink.py --no-cpu > gpurun_out/abt_${v}_$i.log 2>&1 || exit $?
  done
done
