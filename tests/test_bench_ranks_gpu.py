"""bench.py's N-rank path end to end on one GPU: `bench.py --gpus 2` through
torch.distributed.run with every rank on device 0 and gloo in place of RCCL
(SHADOWTOPO_BENCH_ONE_GPU, which RCCL cannot do: it refuses two ranks on one device).  The
launcher, the source sharding, the packed (dense) row codec, the exchange, the barriers and
the rank-0 report all run as on N GPUs; each rank then checks the matrix the exchange
assembled against the whole matrix its own engine computes, bit for bit (bench.rehearsal_check).
A small C2 (scale 0.1, dense: packed rows) and C4 (scale 0.02, sparse: 16-bit hop
counts) keep it to seconds; the full-size C2 and C4 rehearsals at 2 and 4
ranks are recorded in profiles/r06z2_rank_rehearsal/."""
import json
import os
import signal
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("config,scale,ranks,mode", [("C2", 0.1, 2, "packed"), ("C2", 0.1, 3, "packed"),
                                                     ("C4", 0.02, 2, "hops16")])
def test_bench_rank_rehearsal_assembles_the_exact_matrix(config, scale, ranks, mode):
    env = dict(os.environ, SHADOWTOPO_BENCH_ONE_GPU="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(ranks), "--steps", "2", "--warmup", "1",
           "--config", config, "--scale", str(scale), "--no-north-star", "--no-fresh", "--no-host-rate"]
    # its own process group: a hung run is ended with every rank the launcher started
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=110)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        pytest.fail("the rank rehearsal did not finish in 110 s")
    assert p.returncode == 0, err[-3000:]
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-2000:]
    out = json.loads(lines[-1])
    assert out["n_gpus"] == ranks and "rehearsal" in out
    chk = out["rehearsal_check"]
    assert chk["lat_equal"] and chk["rel_equal"] and chk["hops_equal"], chk
    assert chk["ranks_equal"] == [True] * ranks, chk
    assert out["exchange"]["mode"] == mode, out["exchange"]
    assert sum(out["sharding"]["per_rank_rows"]) == out["config"]["attached"], out["sharding"]
