#!/bin/bash
# Session r3 s1: GOST / MD5 kernel times and the ragged-path baseline.
set -u
timeout -k 10 200 python tools/kbench.py --alg md5,gost256,gost512 --reps 30 || exit $?
timeout -k 10 300 python tools/pkt_bench.py --steps 10 || exit $?
