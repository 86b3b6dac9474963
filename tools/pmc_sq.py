"""Per-kernel means of the SQ counters in rocprofv3 counter_collection.csv
files (this library's kernels only), with the derived wave lifetime split.
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
(MI355X_MICROARCH.md); the derived columns are per wave, in cycles."""
import collections
import csv
import re
import sys

OURS = re.compile(r"\bk_\w+")


def main(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                m = OURS.search(r["Kernel_Name"])
                if not m:
                    continue
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, ctr in sorted(acc.items()):
        mean = {k: sum(v) / len(v) for k, v in ctr.items()}
        line = [f"{name:40s}"] + [f"{k}={v:.4g}" for k, v in sorted(mean.items())]
        waves = mean.get("SQ_WAVES", 0)
        if waves:
            for k in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in mean:
                    line.append(f"{k}/wave(cyc)={4 * mean[k] / waves:.0f}")
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS"):
                if k in mean:
                    line.append(f"{k}/wave={mean[k] / waves:.0f}")
        print(" ".join(line))


if __name__ == "__main__":
    main(sys.argv[1:])
