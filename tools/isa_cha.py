"""Instruction mix of the ChaCha block kernels (hipcc -S), for review."""
import re
import subprocess
import sys

src = "liblcb_amd/csrc/chacha_kernels.hip"
extra = sys.argv[1:]
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                       "-S", "-o", "/tmp/cha.s", src] + extra)
s = open("/tmp/cha.s").read()
for m in re.finditer(r"^(_ZN6lcbgpu\d+chacha_\w*kernel\w*):", s, re.M):
    end = s.index("s_endpgm", m.start())
    lines = [l.strip() for l in s[m.start():end].splitlines()[1:]]
    lines = [l for l in lines if l and not l.startswith((".", ";")) and not l.endswith(":")]
    ops = {}
    for l in lines:
        ops[l.split()[0]] = ops.get(l.split()[0], 0) + 1
    valu = sum(v for k, v in ops.items() if k.startswith("v_"))
    print(m.group(1), "instr", len(lines), "valu", valu, "dpp-folded",
          sum(1 for l in lines if "quad_perm" in l and not l.startswith("v_mov")),
          "dpp-mov", ops.get("v_mov_b32_dpp", 0), "s_nop", ops.get("s_nop", 0),
          "alignbit", ops.get("v_alignbit_b32", 0))
