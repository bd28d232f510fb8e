set -o pipefail
O=gpurun_out/s14; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_packets.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "packets or ragged or c4 or keyed" > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab_inproc.py --libs product,head,recs --work fixed,r1k,pkt,c4 --alg md5 --rounds 12 > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu $O/ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/ab_inproc.py --libs product,fw1,fw2 --work fixed --alg md5,sha1 --rounds 12 > $O/ab_fw.txt 2>&1; rc=$?; grep -v amdgpu $O/ab_fw.txt; exit $rc
