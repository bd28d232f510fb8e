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
  # alternate the two builds REPS times, keep each algorithm's best rate
  # (the build container's CPU is shared: single runs swing by 30 %)
  : > $T/ref_all.txt; : > $T/our_all.txt
  for k in $(seq ${REPS:-5}); do $T/ref $N >> $T/ref_all.txt; $T/our $N >> $T/our_all.txt; done
  for w in ref our; do
    awk '{ if (!($1 in best) || $2 > best[$1]) { best[$1] = $2; sum[$1] = $3 } if (!($1 in ord)) { ord[$1] = NR; names[NR] = $1 } }
         END { for (i = 1; i <= NR; i++) if (i in names) print names[i], best[names[i]], sum[names[i]] }' $T/${w}_all.txt > $T/$w.txt
  done
  echo "== $mode build (gcc -O2 $F), 1 KiB messages, one thread, best of ${REPS:-5} alternating runs; $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2)"
  paste $T/ref.txt $T/our.txt | awk '{ printf "%-8s reference %8.1f MiB/s  drop-in %8.1f MiB/s  ratio %.2f  %s\n", $1, $2, $5, $5/$2, ($3==$6)?"same digests":"DIGESTS DIFFER" }'
done
rm -rf $T
