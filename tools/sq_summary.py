"""MFMA-utilisation summary of the dominant conv_gemm8 instances from rocprofv3 PMC passes
(one rocprofv3 --pmc pass per counter group, --kernel-include-regex conv_gemm8; see tools/pmc_g8.sh).

    python tools/sq_summary.py out.json sq1/run_counter_collection.csv sq2/... sq3/...

Units (MI355X_MICROARCH.md): GRBM_GUI_ACTIVE is summed over the 8 XCDs (kernel cycles =
value / 8); SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over every SIMD (32 per
v_mfma_f32_32x32x16_bf16), so MFMA busy = busy / (1024 SIMDs x kernel cycles);
SQ_INSTS_VALU_MFMA_MOPS_BF16 counts 512-FLOP units; SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles.  Peak: 2.5 PFLOP/s dense bf16 (1024 SIMDs x 1024 FLOP/clk at
2.4 GHz)."""
import collections
import csv
import json
import sys

N_SIMD = 1024


def instance(name):
    if "ILi256ELi256E" in name:
        base = "conv_gemm8_kernel<256,256,2,64,2,2,"
    elif "ILi256ELi128E" in name:
        base = "conv_gemm8_kernel<256,128,4,64,2,2,"
    else:
        return name[:60]
    # OutT follows the NS / PHI arguments (…ELi2ELi2E<OutT>…); round-5 names end with the
    # tap-addressing / stream-K argument TA (…Li0ELi<TA>EEEv)
    out = "bf16" if "ELi2ELi2EDF16b" in name else "float"
    ta = ""
    for v in ("1", "3"):
        if name.endswith(f"Li0ELi{v}EEEvNS_10ConvArgsG8E"):
            ta = f",bf16,0,{v}"
    return f"{base}{out},0,1,8,1{ta}>"


def main():
    out, files = sys.argv[1], sys.argv[2:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            k = instance(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {}
    for k, d in vals.items():
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        e = dict(dispatches=len(d.get("GRBM_GUI_ACTIVE", d[next(iter(d))])),
                 counters={c: round(v) for c, v in avg.items()})
        cyc = avg.get("GRBM_GUI_ACTIVE", 0) / 8
        if cyc:
            e["kernel_cycles"] = round(cyc)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                e["mfma_busy_frac"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * cyc), 4)
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in avg:
            fl = avg["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512
            e["gflop_per_dispatch"] = round(fl / 1e9, 3)
            ns = sum(dur[k]) / len(dur[k])
            e["avg_dispatch_us_under_pmc"] = round(ns / 1e3, 2)
            e["tflops_under_pmc"] = round(fl / ns / 1e3, 1)
            e["frac_of_2500_tflops"] = round(fl / ns / 1e3 / 2500, 4)
            if cyc:
                e["clock_ghz"] = round(cyc / ns, 3)
        if "SQ_WAIT_INST_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
            e["wait_inst_any_frac_of_wave_cycles"] = round(avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"], 4)
        if "SQ_WAIT_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
            e["wait_any_frac_of_wave_cycles"] = round(avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"], 4)
        res[k] = e
    json.dump(dict(source=files, note=__doc__.split("\n\n")[1], instances=res), open(out, "w"), indent=1)
    for k, e in res.items():
        print(k, {a: b for a, b in e.items() if a != "counters"})


if __name__ == "__main__":
    main()
