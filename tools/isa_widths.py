"""Memory-instruction widths, registers and LDS of chosen kernels in the gfx950 device assembly.

Usage (CPU, no GPU needed):
  hipcc -O3 --offload-arch=gfx950 -std=c++17 --cuda-device-only -S -I include \
        -o /tmp/crdt_gfx950.s crdt_amd/csrc/crdt_merge.hip
  python3 tools/isa_widths.py /tmp/crdt_gfx950.s k_flags_back k_scan
Prints, per matching kernel instantiation, the static count of each global / LDS load and store opcode
(the widths a wave issues), with .vgpr_count, .sgpr_count and .group_segment_fixed_size from the metadata.
"""
import collections
import re
import subprocess
import sys


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout
        return out.splitlines()
    except Exception:
        return names


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    s = open(path).read()
    meta = {}
    for m in re.finditer(r"\.group_segment_fixed_size:\s+(\d+).*?\.name:\s+(\S+).*?\.sgpr_count:\s+(\d+).*?"
                         r"\.vgpr_count:\s+(\d+)", s, re.S):
        meta[m.group(2)] = (int(m.group(1)), int(m.group(3)), int(m.group(4)))
    bodies = {}
    for m in re.finditer(r"\n(_Z[^\s:]+):[^\n]*\n(.*?)\n\.Lfunc_end", s, re.S):
        bodies[m.group(1)] = m.group(2)
    names = [n for n in bodies if any(p in n for p in pats)]
    for n, d in zip(names, demangle(names)):
        ops = collections.Counter(re.findall(r"\n\s*((?:global|buffer|ds)_(?:load|store|read|write)\w*)", bodies[n]))
        lds, sg, vg = meta.get(n, (None, None, None))
        d = d.replace("(anonymous namespace)::", "")
        print(f"{d[:110]}\n    vgpr {vg}  sgpr {sg}  lds {lds} B  " +
              "  ".join(f"{k} {v}" for k, v in sorted(ops.items())))


if __name__ == "__main__":
    main()
