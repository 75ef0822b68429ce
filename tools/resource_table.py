"""Registers, spills and occupancy of every kernel in a -Rpass-analysis=kernel-resource-usage
report (make -C 3d-ray-tracer-vulkan_amd asm -> build/resource_usage.txt).

    python tools/resource_table.py [report] [--filter SUBSTRING]
"""
import argparse
import re
import sys


def parse(path):
    rows, cur = {}, None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+(?:\S+:\d+:\d+:\s+)?([\w \[\]/]+?): (\S+) \[", line)
        if m and cur:
            rows[cur][m.group(1).strip()] = m.group(2)
    return rows


def short(name):
    m = re.search(r"(trace_\w+?)I(.*)EEvNS_9TraceArgsE", name)
    if not m:
        return name
    args = re.findall(r"L([bi])(\d+)E", m.group(2))
    return f"{m.group(1)}<{', '.join(('true' if v == '1' else 'false') if t == 'b' else v for t, v in args)}>"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("report", nargs="?", default="3d-ray-tracer-vulkan_amd/build/resource_usage.txt")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    for k, v in parse(a.report).items():
        n = short(k)
        if a.filter not in n:
            continue
        print(f"{n:45s} VGPR {v.get('VGPRs', '?'):>4} spill {v.get('VGPRs Spill', '?'):>3} "
              f"SGPR-spill {v.get('SGPRs Spill', '?'):>3} scratch {v.get('ScratchSize [bytes/lane]', '?'):>3} "
              f"waves/SIMD {v.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    sys.exit(main())
