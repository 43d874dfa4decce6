"""Aggregate a rocprofv3 PC-sampling CSV: samples per instruction (and source line).

    python scripts/pcs_summary.py <pc_sampling csv> <out prefix>
writes <prefix>_by_inst.csv (top instructions), <prefix>_by_line.csv (source lines, when the
build carries line tables) and <prefix>_head.csv (the first raw rows, for the column layout)."""
import collections
import csv
import sys


def main():
    src, pre = sys.argv[1], sys.argv[2]
    by_inst, by_line, total = collections.Counter(), collections.Counter(), 0
    with open(src, newline="") as fh, open(pre + "_head.csv", "w", newline="") as hd:
        rd = csv.DictReader(fh)
        cols = rd.fieldnames
        w = csv.writer(hd)
        w.writerow(cols)
        ci = next((c for c in cols if c.lower() == "instruction"), None)
        cc = next((c for c in cols if "comment" in c.lower()), None)
        co = next((c for c in cols if "offset" in c.lower()), None)
        ck = next((c for c in cols if "kernel" in c.lower() and "name" in c.lower()), None)
        for i, r in enumerate(rd):
            if i < 200:
                w.writerow([r[c] for c in cols])
            if ck and "sqp_kernel" not in (r.get(ck) or "sqp_kernel"):
                continue
            total += 1
            key = (r.get(co, ""), r.get(ci, ""))
            by_inst[key] += 1
            if cc:
                by_line[r.get(cc, "")] += 1
    with open(pre + "_by_inst.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["samples", "share", "offset", "instruction"])
        for (off, ins), n in by_inst.most_common(3000):
            w.writerow([n, f"{n / max(total, 1):.5f}", off, ins])
    with open(pre + "_by_line.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["samples", "share", "line"])
        for ln, n in by_line.most_common(3000):
            w.writerow([n, f"{n / max(total, 1):.5f}", ln])
    print(f"{total} samples; columns: {cols}")


if __name__ == "__main__":
    main()
