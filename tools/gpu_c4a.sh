mkdir -p gpurun_out/c4a
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "half_line or ragged or c4_full or bucketed" > gpurun_out/c4a/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/c4a/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/c4ab.sh build_exp/liblcb_base.so build_exp/liblcb_phdef.so "" > gpurun_out/c4a/ab.log 2>&1
rc=$?; cat gpurun_out/c4a/ab.log; exit $rc
