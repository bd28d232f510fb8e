# LDS-DMA cache policy of the MD5 fixed-stride stream (LCB_LDS_AUX), same-process A/B.
set -o pipefail
mkdir -p gpurun_out/r4i
timeout -k 10 300 python -u tools/ab_inproc.py --libs product,aux0,aux1,aux3,aux18 --work fixed --alg md5 --rounds 12 --launches 40 > gpurun_out/r4i/ab_aux.txt 2>&1
