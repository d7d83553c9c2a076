#!/usr/bin/env python3
"""Offline simulation of the frontier engine's round scheduling (src/device/frontier.h).

Grows leaf-wise trees on binned synthetic Higgs-shape data with a numpy split finder
(gain = G_L^2/H_L + G_R^2/H_R - G^2/H with min_sum_hessian_in_leaf), and replays the
device select's policies: which open nodes a round expands, how many rounds a tree takes,
how many expansions are wasted. The split finder is simplified (no missing-value
directions), which is enough for the scheduling question this script answers.

    python scripts/frontier_policy_sim.py [rows] [num_leaves] [trees]
"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def bin_data(X, max_bin=255):
    B = np.empty(X.shape, dtype=np.uint8)
    for j in range(X.shape[1]):
        qs = np.unique(np.quantile(X[:, j], np.linspace(0, 1, max_bin + 1)[1:-1]))
        B[:, j] = np.searchsorted(qs, X[:, j]).astype(np.uint8)
    return B


class Finder:
    def __init__(self, B, g, h, min_hess=100.0):
        self.B, self.g, self.h, self.mh = B, g, h, min_hess

    def best(self, rows):
        g, h = self.g[rows], self.h[rows]
        G, H = g.sum(), h.sum()
        best = (-np.inf, -1, -1)
        for j in range(self.B.shape[1]):
            b = self.B[rows, j]
            hg = np.bincount(b, weights=g, minlength=256)
            hh = np.bincount(b, weights=h, minlength=256)
            cg, ch = np.cumsum(hg)[:-1], np.cumsum(hh)[:-1]
            ok = (ch >= self.mh) & (H - ch >= self.mh)
            if not ok.any():
                continue
            gain = np.where(ok, cg ** 2 / np.maximum(ch, 1e-12) + (G - cg) ** 2 / np.maximum(H - ch, 1e-12) - G ** 2 / H,
                            -np.inf)
            t = int(np.argmax(gain))
            if gain[t] > best[0]:
                best = (float(gain[t]), j, t)
        return best


def grow(finder, n, L, policy, spec=0, kmax=64, M=4, alpha=1.0):
    """Returns (rounds, expansions, committed splits, hist rows / n, committed-only hist rows / n,
    partitioned rows / n)."""
    nodes = {0: dict(rows=np.arange(n), depth=0, parent=-1, left=None, committed=False)}
    nodes[0]["gain"], nodes[0]["feat"], nodes[0]["thr"] = finder.best(nodes[0]["rows"])
    nxt = 1
    leaves = [0]
    ns = 0
    rounds = 0
    exps = 0
    hist_rows = n  # root histogram
    part_rows = 0
    while True:
        rounds += 1
        # replay
        blocked = None
        while len(leaves) < L:
            li = max(range(len(leaves)), key=lambda i: (nodes[leaves[i]]["gain"], -i))
            c = leaves[li]
            if not nodes[c]["gain"] > 0:
                blocked = None
                break
            if nodes[c]["left"] is None:
                blocked = c
                break
            nodes[c]["committed"] = True
            l = nodes[c]["left"]
            leaves[li] = l
            leaves.append(l + 1)
            ns += 1
        if blocked is None:
            committed_hist = sum(min(len(nodes[d["left"]]["rows"]), len(nodes[d["left"] + 1]["rows"]))
                                 for d in nodes.values() if d["committed"])
            return rounds, exps, ns, round(hist_rows / n, 2), round((n + committed_hist) / n, 2), round(part_rows / n, 2)
        R = L - 1 - ns
        alive = [c for c, d in nodes.items() if d["gain"] > 0 and not d["committed"]]

        def elig(c):
            d = nodes[c]
            if d["left"] is not None or not d["gain"] > 0:
                return False
            if d["depth"] + 1 - M >= 1:
                a = c
                for _ in range(M - 1):
                    a = nodes[a]["parent"]
                return nodes[a]["committed"]
            return True

        el = sorted([c for c in alive if elig(c)], key=lambda c: (c != blocked, -nodes[c]["gain"], c))
        if policy == 0:
            eunc = sum(1 for c, d in nodes.items() if d["left"] is not None and not d["committed"])
            K = max(1, min(kmax, R - eunc + spec))
            chosen = el[:K]
        else:
            gains = sorted((nodes[c]["gain"] for c in alive), reverse=True)
            chosen = []
            for c in el:
                rank = sum(1 for x in gains if x > nodes[c]["gain"])
                if c == blocked or rank < int(alpha * R) + spec:
                    chosen.append(c)
            chosen = chosen[:kmax]
        for c in chosen:
            d = nodes[c]
            rows = d["rows"]
            go = finder.B[rows, d["feat"]] <= d["thr"]
            for k, sub in enumerate((rows[go], rows[~go])):
                cid = nxt + k
                nodes[cid] = dict(rows=sub, depth=d["depth"] + 1, parent=c, left=None, committed=False)
                nodes[cid]["gain"], nodes[cid]["feat"], nodes[cid]["thr"] = finder.best(sub)
            d["left"] = nxt
            hist_rows += min(len(nodes[nxt]["rows"]), len(nodes[nxt + 1]["rows"]))
            part_rows += len(rows)
            nxt += 2
            exps += 1


def main():
    from lambdagap_amd.utils import make_higgs_like

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 63
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    X, y = make_higgs_like(n, seed=7)
    B = bin_data(X)
    score = np.zeros(n)
    for it in range(T):
        p = 1 / (1 + np.exp(-score))
        g, h = p - y, p * (1 - p)
        f = Finder(B, g, h)
        res = {}
        for pol, spec, alpha in ((1, 0, 1.0), (1, 0, 0.5), (1, 0, 0.25)):
            res[(pol, spec, alpha)] = grow(f, n, L, pol, spec, alpha=alpha)
        print(it, {f"p{k[0]}s{k[1]}a{k[2]}": v for k, v in res.items()}, flush=True)
        # advance the score with a crude tree of the root split (keeps gradients moving)
        gain, j, t = f.best(np.arange(n))
        left = B[:, j] <= t
        for m in (left, ~left):
            score[m] -= 0.1 * g[m].sum() / max(h[m].sum(), 1e-9)


if __name__ == "__main__":
    main()
