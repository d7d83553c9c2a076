"""Collective training under a torch.distributed (gloo) process group on CPU: the native host
collectives ride on dist.all_gather through LGBM_NetworkInitWithFunctions (allgather-only
transport), the analogue of the reference's Dask workers wiring a socket mesh."""
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


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, learner, out_dir):
    import sys

    # keep each rank's native stderr (gloo / runtime aborts) for the failure report
    err = os.open(os.path.join(out_dir, f"err{rank}.txt"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
    os.dup2(err, 2)
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path.insert(0, ROOT)
    from lambdagap_amd.parallel import DistributedLGBMClassifier, shard, train_distributed

    mat = np.loadtxt(os.path.join(DATA, "binary.train"))
    X, y = mat[:, 1:], mat[:, 0]
    params = {"objective": "binary", "verbosity": -1, "num_leaves": 15, "min_data_in_leaf": 20}
    if mode == "all":  # every rank holds all rows
        b = train_distributed(params, X, y, 6, tree_learner=learner)
        s = b.model_to_string()
    elif mode == "shard":
        b = train_distributed(params, shard(X), shard(y), 6, tree_learner=learner)
        s = b.model_to_string()
    else:  # sklearn estimator
        clf = DistributedLGBMClassifier(n_estimators=6, num_leaves=15, tree_learner=learner)
        clf.fit(shard(X), shard(y))
        s = clf.booster_.model_to_string()
    with open(os.path.join(out_dir, f"m{rank}.txt"), "w") as f:
        f.write(s)


def _run(world, mode, learner, tmp_path):
    port = _port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_worker, args=(r, world, port, mode, learner, str(tmp_path))) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    if codes != [0] * world:
        logs = {r: open(tmp_path / f"err{r}.txt").read()[-3000:] for r in range(world)
                if os.path.exists(tmp_path / f"err{r}.txt")}
        raise AssertionError(f"exit codes {codes}; stderr tails {logs}")
    ms = [open(tmp_path / f"m{r}.txt").read() for r in range(world)]
    trees = [m.split("end of trees")[0] for m in ms]
    assert all(t == trees[0] for t in trees)
    return ms[0]


@pytest.mark.parametrize("world", [2, 3])
def test_torch_network_data_parallel_matches_serial(lgb, tmp_path, world):
    m = _run(world, "all", "data", tmp_path)
    mat = np.loadtxt(os.path.join(DATA, "binary.train"))
    X, y = mat[:, 1:], mat[:, 0]
    serial = lgb.train({"objective": "binary", "verbosity": -1, "num_leaves": 15, "min_data_in_leaf": 20 * world},
                       lgb.Dataset(np.vstack([X] * world), np.concatenate([y] * world)), 6)
    t = np.loadtxt(os.path.join(DATA, "binary.test"))
    np.testing.assert_allclose(lgb.Booster(model_str=m).predict(t[:, 1:]), serial.predict(t[:, 1:]), rtol=1e-6,
                               atol=1e-8)


@pytest.mark.parametrize("learner", ["voting", "feature"])
def test_torch_network_other_learners(lgb, tmp_path, learner):
    m = _run(2, "shard" if learner == "voting" else "all", learner, tmp_path)
    t = np.loadtxt(os.path.join(DATA, "binary.test"))
    from sklearn.metrics import roc_auc_score

    assert roc_auc_score(t[:, 0], lgb.Booster(model_str=m).predict(t[:, 1:])) > 0.67


def test_distributed_sklearn_estimator(lgb, tmp_path):
    m = _run(2, "sklearn", "data", tmp_path)
    t = np.loadtxt(os.path.join(DATA, "binary.test"))
    from sklearn.metrics import roc_auc_score

    assert roc_auc_score(t[:, 0], lgb.Booster(model_str=m).predict(t[:, 1:])) > 0.68


@pytest.mark.parametrize("world", [2, 3])
def test_torch_network_sharded_matches_socket_mesh(lgb, tmp_path, world):
    """Different rows on every rank: the allgather-derived reduce-scatter must reduce each rank's own
    block (identical shards, as in the "all" test above, cannot tell whose block is whose). The
    socket mesh's native reduce-scatter on the same shards is the reference."""
    import sys

    sys.path.insert(0, os.path.dirname(__file__))
    from test_distributed import _run as socket_run

    (tmp_path / "t").mkdir()
    (tmp_path / "s").mkdir()
    m = _run(world, "shard", "data", tmp_path / "t")
    ms = socket_run("data", "split", tmp_path / "s", {"min_data_in_leaf": 20}, world=world)
    t = np.loadtxt(os.path.join(DATA, "binary.test"))
    np.testing.assert_allclose(lgb.Booster(model_str=m).predict(t[:, 1:]),
                               lgb.Booster(model_str=ms[0]).predict(t[:, 1:], num_iteration=6), rtol=1e-6, atol=1e-8)
