"""Reduce tools/pmc_sq.sh's rocprofv3 counter CSVs to per-kernel means (JSON) and the derived wave-
cycle split (MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles,
WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES).
usage: python tools/sq_summary.py OUTDIR/sq1 OUTDIR/sq2 out.json"""
import collections
import csv
import json
import sys


def main():
    *dirs, out = sys.argv[1:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            name = name.split("(")[0].split("<")[0]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        w = m.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in m:
                    m[c + "_frac"] = m[c] / w
        if m.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in m:
            m["lds_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        res[k] = m
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k in ("k_chanfilt_r", "k_chanfilt", "k_etsi_viterbi"):
        if k in res:
            print(k, {c: round(v, 3) for c, v in res[k].items() if c.endswith("_frac")})


if __name__ == "__main__":
    main()
