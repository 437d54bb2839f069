"""bench.py's process launch (CPU, gloo): ``--gpus N`` without WORLD_SIZE starts N ranks
itself; the JSON line reports the world size the process group saw and every rank."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          env=e, timeout=240, cwd=ROOT)


def _line(p):
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (p.stdout, p.stderr[-2000:])
    return json.loads(lines[0])


def test_launcher_starts_two_ranks():
    p = _run(["--gpus", "2", "--stub", "--steps", "3", "--warmup", "1", "--prewarm-s", "0.05"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = _line(p)
    assert out["n_gpus"] == 2 and out["world_size"] == 2
    assert [r["rank"] for r in out["ranks"]] == [0, 1]
    assert len({r["pid"] for r in out["ranks"]}) == 2  # two processes, not one


def test_single_rank_stub():
    p = _run(["--gpus", "1", "--stub", "--steps", "3", "--warmup", "1", "--prewarm-s", "0.05"])
    assert p.returncode == 0, p.stderr[-2000:]
    out = _line(p)
    assert out["n_gpus"] == 1 and len(out["ranks"]) == 1


def test_world_size_mismatch_fails():
    p = _run(["--gpus", "2", "--stub", "--steps", "1", "--warmup", "0", "--prewarm-s", "0"],
             env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in (p.stderr + p.stdout)


def test_mfma_mode_is_config5_only():
    """--mode mfma names the config-5 matrix-core pass; any other config refuses it before
    touching the GPU (C5's mode="fast" runs the exact kernel)."""
    p = _run(["--mode", "mfma", "--config", "c2", "--stub"])
    assert p.returncode != 0
    assert "--mode mfma" in (p.stderr + p.stdout)


def test_rank_parity_checker_on_host_outputs():
    """bench.rank_parity (each rank's own-shard check on N > 1 lines) against the restatement's
    own outputs: equal -> all_equal; one flipped weight bit -> not (CPU, no GPU)."""
    import types

    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    import bench
    from oracle import oracle as orc

    offsets, sid, prob, rel, conf, present = bench.make_c2(300, 32, 500, seed=4)
    cpu = orc.consensus_csr(offsets, sid, prob, rel, conf, present)
    res = types.SimpleNamespace(**{k: torch.from_numpy(np.array(v)) for k, v in cpu.items()})
    ok = bench.rank_parity(res, offsets, sid, prob, rel, conf, present, True, 1, m_sample=200)
    assert ok["all_equal"] and ok["markets"] == 200 and ok["signals"] == 6400
    res.weight[3] = float(np.nextafter(res.weight[3].item(), 2.0))
    assert not bench.rank_parity(res, offsets, sid, prob, rel, conf, present, True, 1, m_sample=200)["all_equal"]
