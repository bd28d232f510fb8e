#!/usr/bin/env python3
"""One-line summary of a tools/pkt_bench.py log: usage pkt_summary.py <tag> <log>."""
import json
import sys

out = []
for line in open(sys.argv[2]):
    if not line.startswith("{"):
        continue
    j = json.loads(line)
    if "ragged_packets" in j:
        out.append("pkt %s" % {k: v["ms_per_pass"] for k, v in j["ragged_packets"].items() if isinstance(v, dict)})
    elif "c4" in j:
        out.append("c4%s %.3f" % (("_" + j["alg"]) if "alg" in j else "", j["c4"]["ms_per_pass"]))
    else:
        out.append("%s%s %s" % (j["variant"], j.get("stride", ""), j["ms"]))
print(sys.argv[1], " | ".join(out))
