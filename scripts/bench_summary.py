#!/usr/bin/env python3
"""One line per bench JSON: the headline figures (device and host-delivered build time,
throughput, roofline fraction, dominant kernel launch time) and, on the default line, the
C4 north-star record."""
import json
import sys

for p in sys.argv[1:]:
    d = json.load(open(p))
    c, r, e = d["config"], d["roofline"], d["engine"]
    print(f"{p}: {c['workload'][:40]} ms/step {d['ms_per_step']:.3f} host {c.get('matrix_build_host_ms') or 0:.3f} "
          f"value {d['value']:.0f} frac {r['frac']:.4f} ({r['bound']}; hbm {(r.get('hbm') or r).get('frac') or 0:.4f}, "
          f"step {(r.get('hbm') or r).get('frac_step') or 0:.4f}) kernel {r['kernel']} {r['avg_launch_ms']:.3f} ms "
          f"rounds {e['rounds_per_step']:.1f} cold {e['cold_start_ms']:.1f} ms fresh {c.get('matrix_build_fresh_ms') or 0:.3f} "
          f"compose {e.get('compose_kernel_ms_per_step') or 0:.3f} ms")
    n = d.get("north_star")
    if n and "matrix_build_ms" in n:
        pr = n.get("projection") or {}
        print(f"  north C4: {n['matrix_build_ms']:.2f} ms host {n.get('matrix_build_host_ms', 0):.2f} ms "
              f"frac {n['roofline']['frac']:.4f} proj " +
              " ".join(f"{k}:{v['per_gpu_ms']:.1f}/{v.get('per_gpu_host_ms', 0):.1f}" for k, v in pr.items()) +
              f" fresh {n.get('matrix_build_fresh_ms') or 0:.2f} compose {n.get('compose_kernel_ms') or 0:.3f}")
        vl = n.get("vertex_loss_variant")
        if vl:
            print(f"  C4L: {vl.get('matrix_build_ms', 0):.2f} ms compose {vl.get('compose_kernel_ms', 0):.3f} ms "
                  f"(no loss {vl.get('compose_kernel_ms_no_loss') or 0:.3f}, ratio {vl.get('compose_ratio') or 0:.2f})")
    elif n:
        print("  north:", n)
