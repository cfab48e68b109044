#!/usr/bin/env python3
"""C2 with OPT_PROFILE: rows the sweep's f32 filter logged (exact-pass rows, stats 'visits')."""
import sys
sys.path.insert(0, ".")
from shadow_amd import engine as E  # noqa: E402
from shadow_amd import synth  # noqa: E402
g = synth.geometric_complete_ish(V=10_000, A=1_000)
eng = E.Engine.from_synth(g)
eng.set_attached(g.attached)
eng.set_option(E.OPT_PROFILE, 1)
eng.compute_rows(want_kind=False)
eng.reset_stats()
eng.compute_rows(want_kind=False)
st = eng.stats()
print({k: st[k] for k in ("visits", "changes", "full_sweeps", "delta_sweeps", "rounds", "full_changes")})
