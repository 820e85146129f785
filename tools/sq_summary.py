"""Summarise one SQ PMC pass (tools/profile_round.sh / tools/gpu_pmc.sh) per
kernel: fractions of wave cycles parked (SQ_WAIT_ANY: s_waitcnt / barrier),
issue-stalled (SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY; VALU part),
VALU instructions per wave, LDS bank-conflict cycles per wave cycle.  The SQ
cycle counters are in quad-cycles (MI355X_MICROARCH.md); the ratios below are
taken between counters of the same unit."""
import collections
import csv
import re
import sys


def main(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for row in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", row["Kernel_Name"]).strip()
        acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
    print(f"{'kernel':36s} {'waves':>8s} {'parked':>7s} {'stalled':>7s} {'issuing':>7s} {'VALU':>6s} "
          f"{'VALU/wave':>9s} {'LDS conf':>8s}")
    for name, c in acc.items():
        cyc = c.get("SQ_WAVE_CYCLES", 0.0)
        waves = c.get("SQ_WAVES", 0.0)
        if not cyc or not waves:
            continue
        f = lambda k: c.get(k, 0.0) / cyc
        print(f"{name[:36]:36s} {waves:8.0f} {f('SQ_WAIT_ANY'):7.2f} {f('SQ_WAIT_INST_ANY'):7.2f} "
              f"{f('SQ_ACTIVE_INST_ANY'):7.2f} {f('SQ_ACTIVE_INST_VALU'):6.2f} "
              f"{c.get('SQ_INSTS_VALU', 0.0) / waves:9.0f} {f('SQ_LDS_BANK_CONFLICT'):8.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
