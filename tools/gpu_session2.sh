set -o pipefail
O=gpurun_out/s21; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_packets.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c4 or c3 or fixed or ragged or gost or sha512 or packets" > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab_inproc.py --libs product,lp0 --work fixed,c4 --alg sha512,gost256 --rounds 6 > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu $O/ab.txt; exit $rc
