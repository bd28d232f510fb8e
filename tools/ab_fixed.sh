LCB_HASH_GPU_LIB=$PWD/build_exp/L.so timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_L.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_L.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do for v in G L; do echo "== $v"; LCB_HASH_GPU_LIB=$PWD/build_exp/$v.so timeout -k 10 100 python3 tools/ramp.py 1 12 | tail -3 || exit 1; LCB_HASH_GPU_LIB=$PWD/build_exp/$v.so timeout -k 10 100 python3 tools/ramp.py 2 12 | tail -2 || exit 1; done; done
