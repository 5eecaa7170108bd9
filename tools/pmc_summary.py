"""Per-kernel HBM traffic from the two rocprofv3 PMC passes of tools/gpu_pmc.sh.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts
half the bytes of a wide coalesced read (MI355X_MICROARCH.md, HBM section), so
the read bytes are reported as 2 x FETCH_SIZE; WRITE_SIZE is taken as is.
Usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> [kernel-substring] [--json out.json]
"""
import csv
import json
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            per[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]))
    return per


def main():
    base = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    fetch = load(f"{base}_fetch/run_counter_collection.csv")
    write = load(f"{base}_write/run_counter_collection.csv")
    out = {}
    for name in sorted(set(fetch) | set(write), key=lambda k: -sum(fetch.get(k, [0]))):
        if want and want not in name:
            continue
        f, w = fetch.get(name, []), write.get(name, [])
        if not f or not w:
            continue
        rd = 2 * 1024 * sum(f) / len(f)
        wr = 1024 * sum(w) / len(w)
        out[name] = dict(launches=len(f), read_bytes=rd, write_bytes=wr, traffic_bytes=rd + wr)
        print(f"{len(f):6d} read {rd / 1e6:9.3f} MB  write {wr / 1e6:9.3f} MB  per launch  {name}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
