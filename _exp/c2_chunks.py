"""Staged-chunk fraction and sweep time of the pruned C2 sweep on the GPU (OPT_SWEEP_STATS,
OPT_TIMING), per option setting: `name=value` pairs of engine options, settings separated by
'/'.  The first computation of each setting warms the heavy-first order; the next ones are
reported.  Compare with the offline floors of _exp/chunk_plane_sim.py (final thresholds).
usage: python3 _exp/c2_chunks.py [scale] ["sweep_windows=8 / sweep_windows=4104 / ..."] [reps] [computations]"""
import sys

sys.path.insert(0, '.')
from shadow_amd import engine as E
from shadow_amd import synth

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 2
N = int(sys.argv[4]) if len(sys.argv) > 4 else 5
settings = [x.split() for x in (sys.argv[2] if len(sys.argv) > 2 else "").split("/")]
g = synth.geometric_complete_ish(V=int(10_000 * scale), A=int(1_000 * scale))
eng = E.Engine.from_synth(g)
eng.set_attached(g.attached)
eng.set_option(E.OPT_TIMING, 1)
for rep in range(REPS):
    for opts in settings:
        for kv in opts:
            k, v = kv.split("=")
            eng.set_option(getattr(E, "OPT_" + k.upper()), int(v))
        eng.set_option(E.OPT_SWEEP_STATS, 0)
        eng.compute_rows(want_kind=False)
        eng.reset_stats()
        for _ in range(N):
            eng.compute_rows(want_kind=False)
        t = eng.stats()
        eng.set_option(E.OPT_SWEEP_STATS, 1)
        eng.reset_stats()
        eng.compute_rows(want_kind=False)
        st = eng.stats()
        print(f"rep {rep} {' '.join(opts) or 'default'}: staged {st['sweep_chunks'] / max(1, st['sweep_chunk_slots']):.4f} "
              f"of block-chunks, {st['sweep_hit_rows']} logged rows ({st['sweep_hit_rows'] / max(1, st['sweep_chunk_slots'] // 313 * 4):.1f} per wave); sweep {t['full_ms'] / max(1, t['full_sweeps']):.3f} ms, delta {t['delta_ms'] / N:.3f} ms, "
              f"wall {t['wall_ms'] / N:.3f} ms per computation", flush=True)
        eng.set_option(E.OPT_SWEEP_WINDOWS, 8)
        eng.set_option(E.OPT_SWEEP_GLDS, 0)
        eng.set_option(E.OPT_SWEEP_WAVES, 4)
        eng.set_option(E.OPT_SWEEP_REFILTER, 0)
        eng.set_option(E.OPT_SWEEP_PARTS, 2)
        eng.set_option(E.OPT_DENSE_BATCHES_PER_WAVE, 1)
eng.close()
