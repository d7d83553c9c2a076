"""Multi-process distributed training on CPU over the TCP socket mesh (2 ranks, 127.0.0.1).

Covers the three parallel tree learners (data / feature / voting) and the
distributed bin-finding path, the CPU analogue of the reference's
examples/parallel_learning setup.
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

# socket meshes and gloo rendezvous pick free localhost ports: under pytest-xdist run these
# modules in one worker (--dist loadgroup) so two tests never race for the same port
pytestmark = pytest.mark.xdist_group("localhost-network")

DATA = os.path.join(os.path.dirname(__file__), "data")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_ports(n):
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def _worker(rank, ports, learner, rows, out_dir, extra):
    world = len(ports)
    import sys

    sys.path.insert(0, ROOT)
    import lambdagap_amd as lgb

    mat = np.loadtxt(os.path.join(DATA, "binary.train"))
    X, y = mat[:, 1:], mat[:, 0]
    if rows == "split":
        X, y = X[rank::world], y[rank::world]
    machines = ",".join(f"127.0.0.1:{p}" for p in ports)
    params = {"objective": "binary", "tree_learner": learner, "num_machines": world, "machines": machines,
              "local_listen_port": ports[rank], "verbosity": -1, "num_leaves": 15, "pre_partition": True,
              "time_out": 2, **extra}
    b = lgb.train(params, lgb.Dataset(X, y, params=params), 8)
    with open(os.path.join(out_dir, f"model{rank}.txt"), "w") as f:
        f.write(b.model_to_string())


def _run(learner, rows, tmp_path, extra=None, world=2):
    ports = _free_ports(world)
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, ports, learner, rows, str(tmp_path), extra or {}))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    return [open(tmp_path / f"model{r}.txt").read() for r in range(world)]


def _trees(s):
    return s.split("end of trees")[0]


@pytest.mark.parametrize("learner,world", [("data", 2), ("voting", 2), ("data", 3), ("voting", 3)])
def test_row_sharded_learners(lgb, tmp_path, learner, world):
    ms = _run(learner, "split", tmp_path, world=world)
    m0 = ms[0]
    # every rank ends with the same model
    assert all(_trees(m) == _trees(m0) for m in ms)
    b = lgb.Booster(model_str=m0)
    t = np.loadtxt(os.path.join(DATA, "binary.test"))
    from sklearn.metrics import roc_auc_score

    assert roc_auc_score(t[:, 0], b.predict(t[:, 1:])) > 0.75


@pytest.mark.parametrize("world", [2, 3, 4])
def test_data_parallel_matches_serial_on_same_bins(lgb, tmp_path, world):
    """Every rank holding ALL rows: data-parallel sums `world` identical copies of every histogram (through
    recursive halving / doubling for 2 and 4 ranks, ring + Bruck for 3), which is the serial histogram of
    the rows repeated `world` times -> the same model."""
    ms = _run("data", "all", tmp_path, {"min_data_in_leaf": 20}, world=world)
    m0 = ms[0]
    assert all(_trees(m) == _trees(m0) for m in ms)
    mat = np.loadtxt(os.path.join(DATA, "binary.train"))
    X, y = mat[:, 1:], mat[:, 0]
    serial = lgb.train({"objective": "binary", "verbosity": -1, "num_leaves": 15, "min_data_in_leaf": 20 * world},
                       lgb.Dataset(np.vstack([X] * world), np.concatenate([y] * world)), 8)
    t = np.loadtxt(os.path.join(DATA, "binary.test"))
    np.testing.assert_allclose(lgb.Booster(model_str=m0).predict(t[:, 1:]), serial.predict(t[:, 1:]), rtol=1e-6,
                               atol=1e-8)


def test_feature_parallel_matches_serial(lgb, tmp_path):
    m0, m1 = _run("feature", "all", tmp_path)
    assert _trees(m0) == _trees(m1)
    mat = np.loadtxt(os.path.join(DATA, "binary.train"))
    serial = lgb.train({"objective": "binary", "verbosity": -1, "num_leaves": 15}, lgb.Dataset(mat[:, 1:], mat[:, 0]),
                       8)
    t = np.loadtxt(os.path.join(DATA, "binary.test"))
    np.testing.assert_allclose(lgb.Booster(model_str=m0).predict(t[:, 1:]), serial.predict(t[:, 1:]), rtol=1e-9)


def _ft_worker(rank, ports, out_dir, fault, init_model, rounds):
    """Data-parallel worker that checkpoints its model text after every iteration."""
    import sys

    if fault:
        os.environ["LGAP_FAULT_INJECT"] = fault
    sys.path.insert(0, ROOT)
    import lambdagap_amd as lgb

    world = len(ports)
    mat = np.loadtxt(os.path.join(DATA, "binary.train"))
    X, y = mat[rank::world, 1:], mat[rank::world, 0]
    machines = ",".join(f"127.0.0.1:{p}" for p in ports)
    params = {"objective": "binary", "tree_learner": "data", "num_machines": world, "machines": machines,
              "local_listen_port": ports[rank], "verbosity": -1, "num_leaves": 15, "pre_partition": True,
              "time_out": 1, "seed": 3}

    def checkpoint(env):
        # every rank holds the identical model: each writes its own snapshot atomically
        path = os.path.join(out_dir, f"ckpt{rank}.txt")
        env.model.save_model(path + ".tmp")
        os.replace(path + ".tmp", path)

    b = lgb.train(params, lgb.Dataset(X, y, params=params), rounds, init_model=init_model, callbacks=[checkpoint])
    with open(os.path.join(out_dir, f"model{rank}.txt"), "w") as f:
        f.write(b.model_to_string())


def _run_ft(tmp_path, fault=None, init_models=None, rounds=8, world=2, join_s=120):
    ports = _free_ports(world)
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_ft_worker, args=(r, ports, str(tmp_path), fault,
                                                  init_models[r] if init_models else None, rounds))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=join_s)
    alive = [p.is_alive() for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    return [p.exitcode for p in procs], alive


def test_fault_injection_peer_exit_is_detected_and_training_resumes(lgb, tmp_path):
    """a rank that dies mid-training (LGAP_FAULT_INJECT) must make its peers fail
    promptly instead of hanging; relaunching every rank from its last checkpoint (init_model) finishes
    the job with the same trees as an uninterrupted run."""
    ref_dir = tmp_path / "ref"
    ref_dir.mkdir()
    codes, _ = _run_ft(ref_dir)
    assert codes == [0, 0], codes
    ref = open(ref_dir / "model0.txt").read()

    run_dir = tmp_path / "run"
    run_dir.mkdir()
    codes, alive = _run_ft(run_dir, fault="1:4:exit")
    assert not any(alive), "a peer of the failed rank hung instead of failing"
    assert codes[1] == 3, codes              # the injected exit
    assert codes[0] not in (0, None), codes  # the survivor raised instead of finishing
    ckpts = [str(run_dir / f"ckpt{r}.txt") for r in range(2)]
    done = [lgb.Booster(model_file=c).num_trees() for c in ckpts]
    assert done[1] == 4 and done[0] >= 4, done

    # resume both ranks from rank 1's last snapshot (the one every rank reached)
    codes, _ = _run_ft(run_dir, init_models=[ckpts[1], ckpts[1]], rounds=8 - done[1])
    assert codes == [0, 0], codes
    resumed = open(run_dir / "model0.txt").read()
    assert lgb.Booster(model_str=resumed).num_trees() == 8
    assert _trees(resumed).split("Tree=")[1:] == _trees(ref).split("Tree=")[1:]


def test_fault_injection_throw_propagates(lgb, tmp_path):
    """mode "throw": the failing rank raises through the normal error path; its peer fails too."""
    codes, alive = _run_ft(tmp_path, fault="0:2:throw")
    assert not any(alive)
    assert all(c not in (0, None) for c in codes), codes
