"""Summarise tools/diag/g2_pmc.sh output: per run, the hipps kernel's SQ counters summed over its
dispatches, as shares of SQ_WAVE_CYCLES (waiting on any instruction / on LDS, issuing), and MFMA
busy cycles relative to 4 x SQ_BUSY_CYCLES (the ratio rocprofv3's MFMA-utilisation metrics use
per SIMD; read it as a relative number across kernels)."""
import csv
import glob
import os
import sys


def main(d):
    for run in sorted(os.listdir(d)):
        files = glob.glob(os.path.join(d, run, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        tot = {}
        for f in files:
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                if "hipps" not in name:
                    continue
                c = r["Counter_Name"]
                tot[c] = tot.get(c, 0.0) + float(r["Counter_Value"])
        if not tot:
            continue
        wc = tot.get("SQ_WAVE_CYCLES", 0) or 1
        bc = tot.get("SQ_BUSY_CYCLES", 0) or 1
        t = open(os.path.join(d, run + ".time")).read().strip() if os.path.exists(os.path.join(d, run + ".time")) else ""
        print(f"{run:10s} wait_inst_any/wave {tot.get('SQ_WAIT_INST_ANY', 0) / wc:6.1%}  "
              f"wait_any/wave {tot.get('SQ_WAIT_ANY', 0) / wc:6.1%}  "
              f"wait_inst_lds/wave {tot.get('SQ_WAIT_INST_LDS', 0) / wc:6.1%}  "
              f"active_inst/wave {tot.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.1%}  "
              f"mfma_busy/(busy*4) {tot.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (4 * bc):6.1%}  "
              f"lds_bank_conflict {tot.get('SQ_LDS_BANK_CONFLICT', 0):.3g}  | {t}")


if __name__ == "__main__":
    main(sys.argv[1])
