"""bench.py contract: `python bench.py --gpus N` outside torchrun launches N rank processes
itself (torch.distributed.run, 127.0.0.1 rendezvous) and relays exactly one JSON line from
rank 0, as the driver's multi-GPU scaling run invokes it. The CPU learner over gloo stands in
for the GPUs here."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_spawns_ranks_and_relays_rank0_line():
    out = _run(["--gpus", "2", "--device", "cpu", "--rows", "20000", "--valid-rows", "4000", "--steps", "2",
                "--warmup", "1"])
    assert out["n_gpus"] == 2
    assert out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["transport"] == "gloo (host collectives)"
    assert out["value"] > 0 and 0.5 < out["auc"] <= 1.0


def test_bench_single_process_cpu():
    out = _run(["--device", "cpu", "--rows", "20000", "--valid-rows", "4000", "--steps", "2", "--warmup", "1"])
    assert out["n_gpus"] == 1 and out["config"]["transport"] is None
    for key in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype", "data"):
        assert key in out
