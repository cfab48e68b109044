#!/usr/bin/env python3
"""LDS occupancy of a kernel from one rocprofv3 --pmc pass (SQ_LDS_IDX_ACTIVE,
SQ_LDS_BANK_CONFLICT, SQ_INSTS_LDS, SQ_WAVES, GRBM_GUI_ACTIVE): per dispatch of the kernels
matching KERNEL_RE, the last N of them averaged.  SQ_LDS_IDX_ACTIVE counts LDS-array cycles
(MI355X_MICROARCH.md, LDS); the CU-cycles available are GRBM_GUI_ACTIVE / 8 (the sum over
the 8 XCDs) x 256 CUs; SQ counters cover a sample of waves, scaled by Grid_Size / 64 over
SQ_WAVES as in roofline_counters.py.  usage: lds_counters.py PMC_DIR KERNEL_RE N"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from roofline_counters import dispatches  # noqa: E402

d, kre, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
ds = dispatches(d, kre)[-n:]
rows = []
for x in ds:
    scale = (x["_grid"] / 64) / max(1.0, x.get("SQ_WAVES", 0.0))
    cu_cycles = x.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 256
    lds = x.get("SQ_LDS_IDX_ACTIVE", 0.0) * scale
    rows.append({"ms": x["_ns"] / 1e6, "wave_scale": scale, "lds_idx_active": lds,
                 "lds_bank_conflict": x.get("SQ_LDS_BANK_CONFLICT", 0.0) * scale,
                 "insts_lds": x.get("SQ_INSTS_LDS", 0.0) * scale, "cu_cycles": cu_cycles,
                 "lds_busy_frac": lds / cu_cycles if cu_cycles else None,
                 "lds_busy_frac_if_quad": 4 * lds / cu_cycles if cu_cycles else None})
avg = {k: sum(r[k] for r in rows) / len(rows) for k in rows[0] if rows[0][k] is not None}
print(json.dumps({"kernel_re": kre, "dispatches": len(rows), "avg": avg}, indent=1))
