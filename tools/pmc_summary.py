"""Per-kernel MFMA utilisation from a rocprofv3 --pmc counter_collection.csv
(tools/pmc_learner.sh): counters averaged per (kernel, grid size), kernel
duration from the dispatch's Start/End timestamps, and

  mfma_util_chip  = SQ_VALU_MFMA_BUSY_CYCLES / (duration x 2.4 GHz x 1024 SIMDs)
  mfma_util_wgs   = the same over the SIMDs the grid can occupy
                    (min(1024, 4 x workgroups x waves_per_wg / 4))

SQ_VALU_MFMA_BUSY_CYCLES counts cycles (32 per 32x32x16 bf16 MFMA, 64 per
32x32x2 f32), SQ_WAVE_CYCLES / SQ_WAIT_INST_ANY count quad-cycles
(/opt/skills/guides/MI355X_MICROARCH.md).

    python3 tools/pmc_summary.py gpurun_out/pmcl/u/pmc_counter_collection.csv ... > profiles/X.json"""
import collections
import csv
import json
import re
import sys

CLK = 2.4e9
SIMDS = 1024


def main(paths):
    out = []
    for path in paths:
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        dur = collections.defaultdict(dict)
        meta = {}
        for r in csv.DictReader(open(path)):
            name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
            if "at::native" in r["Kernel_Name"] or "rocclr" in name:
                continue
            key = (name, int(r["Grid_Size"]))
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            meta[key] = dict(workgroup=int(r["Workgroup_Size"]), vgpr=int(r["VGPR_Count"]),
                             agpr=int(r["Accum_VGPR_Count"]), lds=int(r["LDS_Block_Size"]))
        for key, d in agg.items():
            name, grid = key
            m = {c: sum(v) / len(v) for c, v in d.items()}
            ds = sorted(dur[key].values())
            us = ds[len(ds) // 2] / 1e3
            wg = grid // meta[key]["workgroup"]
            simds = min(SIMDS, wg * max(1, meta[key]["workgroup"] // 64))
            busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
            cyc = us * 1e-6 * CLK
            out.append(dict(source=path, kernel=name, grid=grid, workgroups=wg, **meta[key], dispatches=len(ds),
                            median_us=round(us, 2), counters={c: round(v) for c, v in m.items()},
                            mfma_util_chip=round(busy / (cyc * SIMDS), 4) if cyc else None,
                            mfma_util_wgs=round(busy / (cyc * simds), 4) if cyc else None,
                            valu_insts_per_mfma=round(m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"], 1)
                            if m.get("SQ_INSTS_MFMA") else None))
    print(json.dumps(dict(note=__doc__.split("\n\n")[0], clock_hz=CLK, simds=SIMDS, kernels=out), indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
