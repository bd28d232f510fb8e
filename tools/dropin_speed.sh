#!/bin/bash
# SURVEY.md 8(d) calibration: single-thread MiB/s of the drop-in headers
# (include/crypto/hash) against the reference's headers, same source
# (tests/c/dropin_speed.c), same flags.  Needs /root/reference (build
# container); REF=<dir> overrides.  Prints one table per build mode.
R=$(cd "$(dirname "$0")/.." && pwd)
REF=${REF:-/root/reference}
T=$(mktemp -d)
N=${N:-16384}
for mode in generic simd; do
  if [ $mode = simd ]; then F="-DSPEED_SIMD -msse4.1 -mssse3 -msha -mavx2"; else F=""; fi
  gcc -O2 -w $F -I"$REF/include" -o $T/ref "$R/tests/c/dropin_speed.c" || exit 1
  gcc -O2 -w $F -I"$R/include" -o $T/our "$R/tests/c/dropin_speed.c" || exit 1
  $T/ref $N > $T/ref.txt; $T/our $N > $T/our.txt
  echo "== $mode build (gcc -O2 $F), 1 KiB messages, one thread; $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2)"
  paste $T/ref.txt $T/our.txt | awk '{ printf "%-8s reference %8.1f MiB/s  drop-in %8.1f MiB/s  ratio %.2f  %s\n", $1, $2, $5, $5/$2, ($3==$6)?"same digests":"DIGESTS DIFFER" }'
done
rm -rf $T
