"""DESIGN §6 PMC table from a pmc_sq.json (tools/pmc_kernels.py output): MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (1,024 SIMDs x GRBM_GUI_ACTIVE / 8), VALU = SQ_INSTS_VALU per SIMD-cycle,
conflicts = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, wait = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES.

    python tools/pmc_table.py profiles/rNN/pmc_sq.json [kernel substrings ...]"""
import json
import sys

d = json.load(open(sys.argv[1]))
keys = sys.argv[2:]
for k, v in d.items():
    if keys and not any(s in k for s in keys):
        continue
    g = lambda c: v.get(c, {}).get("mean", 0.0)  # noqa: E731
    simd_cycles = 1024 * g("GRBM_GUI_ACTIVE") / 8
    if not simd_cycles or not g("SQ_LDS_IDX_ACTIVE") or not g("SQ_WAVE_CYCLES"):
        continue
    print(f"{k[:58]:58s} busy {g('SQ_VALU_MFMA_BUSY_CYCLES') / simd_cycles:.3f}  "
          f"valu {g('SQ_INSTS_VALU') / simd_cycles:.3f}  lds-conflict {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f}  "
          f"wait {g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}  dispatches {v['SQ_WAVE_CYCLES']['dispatches']}")
