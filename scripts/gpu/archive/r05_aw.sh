set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05/sanity_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05/sanity_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 400 python -u scripts/sweep_env.py T1 6 '' 'HCLIB_HIP_SPILL_LO=192' 'HCLIB_HIP_SPILL_LO=288' 'HCLIB_HIP_SPILL_LO=352' > gpurun_out/r05/sweep_t1_n.log 2>&1; tail -4 gpurun_out/r05/sweep_t1_n.log
