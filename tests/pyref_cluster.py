"""Independent pure-Python restatement of ReadClusteringEngine::run_clustering after
construct_indices (src/clustering/ReadClusteringEngine.cpp:301-802), written from the
reference text, for small inputs.  Uses the same deterministic orders the C++ engine
documents (host/clustering.h): components by ascending id, connections by (score desc, x, y),
first maximum wins.  Spectral clustering uses numpy.linalg.eigh (Eigen2's
SelfAdjointEigenSolver in the reference) and a port of Evrot / ClusterRotate
(src/lib/clustering/Evrot.cpp, ClusterRotate.cpp).
"""
import math
from collections import deque

import numpy as np


def sort_conns(c):
    return sorted(c, key=lambda t: (-t[2], t[0], t[1]))


def union_find(conns, restricted, min_size, max_size):   # :424-489
    if max_size == -1:
        max_size = 2 ** 31 - 1
    parent, comps, trees, restr = {}, {}, {}, {}
    for x, y, *_ in conns:
        for v in (x, y):
            if v not in parent:
                parent[v] = v
                comps[v] = [v]
                trees[v] = []
                restr[v] = v in restricted

    def find(v):
        path = []
        while parent[v] != v:
            path.append(v)
            v = parent[v]
        for p in path:
            parent[p] = v
        return v

    for x, y, *_ in conns:
        px, py = find(x), find(y)
        if px == py or (restr[px] and restr[py]):
            continue
        if len(comps[px]) + len(comps[py]) > max_size:
            continue
        big, small = (px, py) if len(comps[px]) > len(comps[py]) else (py, px)
        for c in comps[small]:
            parent[c] = big
        comps[big] = comps[big] + comps[small]
        del comps[small]
        trees[big] = trees[big] + [(x, y)] + trees[small]
        del trees[small]
        restr[big] = restr[big] or restr[small]
        del restr[small]
    thr = min_size if min_size >= 0 else 2 ** 64   # int -> size_t comparison
    return [(comps[r], trees[r]) for r in sorted(comps) if len(comps[r]) >= thr]


# ---------------------------------------------------------------- spectral (numpy)
def _build_uab(theta, a, b, ik, jk, D):
    U = np.eye(D)
    for k in range(a, b + 1):
        t = theta[k]
        for i in range(D):
            u = U[i, ik[k]] * math.cos(t) - U[i, jk[k]] * math.sin(t)
            U[i, jk[k]] = U[i, ik[k]] * math.sin(t) + U[i, jk[k]] * math.cos(t)
            U[i, ik[k]] = u
    return U


def _evrot(X):
    N, D = X.shape
    ik = [i for i in range(D - 1) for j in range(i + 1, D)]
    jk = [j for i in range(D - 1) for j in range(i + 1, D)]
    A_ = len(ik)

    def qual(Y):
        Y2 = Y ** 2
        mx = Y2.max(axis=1)
        return 1.0 - ((Y2 / mx[:, None]).sum() / N - 1.0) / D

    def rot(th):
        return X @ _build_uab(th, 0, A_ - 1, ik, jk, D)

    def grad(th, k):
        V = np.zeros((D, D))
        V[ik[k], ik[k]] = -math.sin(th[k])
        V[ik[k], jk[k]] = math.cos(th[k])
        V[jk[k], ik[k]] = -math.cos(th[k])
        V[jk[k], jk[k]] = -math.sin(th[k])
        A = X @ _build_uab(th, 0, k - 1, ik, jk, D) @ V @ _build_uab(th, k + 1, A_ - 1, ik, jk, D)
        Y = rot(th)
        mc = np.abs(Y).argmax(axis=1)
        mv = Y[np.arange(N), mc]
        dJ = 0.0
        for j in range(D):
            for i in range(N):
                dJ += A[i, j] * Y[i, j] / mv[i] ** 2 - A[i, mc[i]] * Y[i, j] ** 2 / mv[i] ** 3
        return 2 * dJ / N / D

    theta = [0.0] * A_
    theta_new = [0.0] * A_
    Q = qual(X)
    q1 = q2 = Q
    it = 0
    while it < 200:
        it += 1
        for d in range(A_):
            theta_new[d] = theta[d] - grad(theta, d)
            qn = qual(rot(theta_new))
            if qn > Q:
                theta[d] = theta_new[d]
                Q = qn
            else:
                theta_new[d] = theta[d]
        if it > 2 and Q - q2 < 1e-3:
            break
        q2, q1 = q1, Q
    Xr = rot(theta_new)
    col = np.abs(Xr).argmax(axis=1)
    clusters = [[i for i in range(N) if col[i] == j] for j in range(D)]
    return Q, clusters, Xr


def _cluster_rotate(X):
    maxq = 0.0
    clusters, vrot = [], None
    vin = X[:, :2].copy()
    e = None
    for g in range(2, X.shape[1] + 1):
        if g > 2:
            vin = np.concatenate([e[2], X[:, g - 1:g]], axis=1)
        e = _evrot(vin)
        if e[0] > maxq:
            maxq = e[0]
        if e[0] > maxq or maxq - e[0] <= 0.001:
            clusters, vrot = [list(c) for c in e[1]], e[2]
    out = []
    for c in clusters:
        if not c:
            out.append([])
            continue
        centre = vrot[c].mean(axis=0)
        d = [((vrot[p] - centre) ** 2).sum() for p in c]
        out.append([p for _, p in sorted(zip(d, c), key=lambda t: t[0])])
    return out


def spectral_clustering(conns, dims):   # :653-697
    to_id, id_to, scores = {}, [], []
    for x, y, s, *_ in conns:
        for v in (x, y):
            if v not in to_id:
                to_id[v] = len(id_to)
                id_to.append(v)
        scores.append(s)
    n = len(id_to)
    mx, mn = max(scores), min(scores)
    if mx == mn:   # scale_strength 0/0 = NaN for every edge (:672-674): every component alone (host/clustering.cpp)
        return [[v] for v in id_to]
    m = np.zeros((n, n))
    for x, y, s, *_ in conns:
        w = math.exp((20 - 0.3) * (s - mn) / (mx - mn) + 0.3)
        m[to_id[x], to_id[y]] = m[to_id[y], to_id[x]] = w
    dims = min(n, dims)
    deg = 1 / np.sqrt(m.sum(axis=1))
    lap = deg[:, None] * m * deg[None, :]
    val, vec = np.linalg.eigh(lap)
    big = np.abs(vec).argmax(axis=0)   # sign convention of host/clustering.cpp sym_eigen
    vec = vec * np.where(vec[big, np.arange(n)] < 0, -1.0, 1.0)[None, :]
    order = np.argsort(-val, kind="stable")
    X = vec[:, order[:dims]]
    return [[id_to[i] for i in c] for c in _cluster_rotate(X)]


# ---------------------------------------------------------------- engine
class Engine:
    def __init__(self, idx, lengths, categories, avg_len, debug, cfg, first_id=1, start=None, end=None):
        self.cfg, self.debug, self.avg_len, self.first_id = cfg, debug, avg_len, first_id
        n = len(lengths)
        self.cat = {first_id + i: int(categories[i]) for i in range(n)}
        self.start = {first_id + i: int(start[i]) if start is not None else 0 for i in range(n)}
        self.end = {first_id + i: int(end[i]) if end is not None else 0 for i in range(n)}
        self.printed = []   # print_components' lines under debug
        hp, sk = idx["hit_ptr"], idx["sorted_kid"]
        self.lengths = {first_id + i: int(l) for i, l in enumerate(lengths)}
        self.comps = {}
        self.pos = {}
        for i in range(len(hp) - 1):
            if hp[i + 1] == hp[i]:
                continue
            rid = first_id + i
            self.comps[rid] = {"reads": [rid], "kmers": [int(v) for v in sk[hp[i]:hp[i + 1]]],
                               "cats": {int(categories[i])}}
            fp = idx["first_ptr"]
            self.pos[rid] = {int(k): int(p) for k, p in zip(idx["first_kid"][fp[i]:fp[i + 1]],
                                                            idx["first_pos"][fp[i]:fp[i + 1]])}
        kp, kr = idx["kci_ptr"], idx["kci_read"]
        self.kci = [[int(v) for v in kr[kp[k]:kp[k + 1]]] for k in range(len(kp) - 1)]

    def good(self, x, y):
        return self.debug and x in self.comps and y in self.comps and self.comps[x]["cats"] == self.comps[y]["cats"]

    def get_connections(self, pivots, min_score):   # :301-333
        out = []
        for p in pivots:
            cnt = {}
            for k in self.comps[p]["kmers"]:
                for c in self.kci[k]:
                    cnt[c] = cnt.get(c, 0) + 1
            cnt.pop(p, None)
            out += [(p, c, s, self.good(p, c)) for c, s in cnt.items() if s >= min_score]
        return sort_conns(out)

    def accumulate(self, ids):
        return sorted({k for i in ids if i in self.comps for k in self.comps[i]["kmers"]})

    def merge(self, components):   # :349-422
        merged, removal = [], {}
        for ids in components:
            if not ids:
                continue
            if len(ids) == 1:
                merged.append(ids[0])
                continue
            cats, reads = set(), []
            for i in ids:
                reads += self.comps[i]["reads"]
                self.comps[i]["reads"] = []
                cats |= self.comps[i]["cats"]
            acc = self.accumulate(ids)
            s = self.comps[ids[0]]
            s["kmers"], s["cats"], s["reads"] = acc, cats, reads
            merged.append(ids[0])
            for i in ids:
                for k in self.comps[i]["kmers"]:
                    removal.setdefault(k, []).append(i)
        for k, rem in removal.items():
            rem.sort()
            lst, upd, i, j = self.kci[k], [], 0, 0
            while i < len(rem) and j < len(lst):
                if rem[i] < lst[j]:
                    i += 1
                elif lst[j] < rem[i]:
                    upd.append(lst[j])
                    j += 1
                else:
                    i += 1
                    j += 1
            self.kci[k] = upd
        return merged

    def remove_merged(self):
        self.comps = {k: v for k, v in self.comps.items() if v["reads"]}

    def ids(self, thr):
        t = thr if thr >= 0 else 2 ** 64
        return [k for k in sorted(self.comps) if len(self.comps[k]["reads"]) >= t]

    def overlap(self, x, y):   # :491-507
        a, b = self.comps[x]["kmers"], self.comps[y]["kmers"]
        i = j = 0
        shared = []
        while i < len(a) and j < len(b):
            if a[i] < b[j]:
                i += 1
            elif b[j] < a[i]:
                j += 1
            else:
                shared.append(a[i])
                i += 1
                j += 1
        if not shared:
            return 0
        xp = [self.pos[x].get(k, 0) for k in shared]
        yp = [self.pos[y].get(k, 0) for k in shared]
        return max(max(xp) - min(xp), max(yp) - min(yp))

    def tails(self, tree):   # :509-573
        adj = {}
        for a, b in tree:
            d = self.overlap(a, b)
            adj.setdefault(a, {}).setdefault(b, d)
            adj.setdefault(b, {}).setdefault(a, d)
        if not adj:
            return [], []
        M = 2 ** 64

        def bfs(start):
            q, vis, dist = deque([start]), set(), {start: self.lengths[start]}
            while q:
                v = q.popleft()
                vis.add(v)
                for a, d in sorted(adj.get(v, {}).items()):
                    if a not in vis:
                        dist[a] = (dist[v] + self.lengths[a] - d) % M
                        q.append(a)
            return dist

        def far(dist):
            best = None
            for k in sorted(dist):
                if best is None or dist[k] > dist[best]:
                    best = k
            return best, dist[best]

        init = bfs(min(adj))
        f, _ = far(init)
        tl = self.avg_len * 2
        dr = bfs(f)
        fr, frd = far(dr)
        right = [v for v in sorted(dr) if (dr[v] + tl) % M > frd]
        dl = bfs(fr)
        fl, fld = far(dl)
        left = [v for v in sorted(dl) if (dl[v] + tl) % M > fld]
        return left, right

    def amplify(self, comp, min_score):
        ids = set(comp)
        for x, y, *_ in self.get_connections(comp, min_score):
            ids |= {x, y}
        return sorted(ids)

    def core_connections(self, cts):   # :586-651
        tails = {}
        for comp, tree in cts:
            l, r = self.tails(tree)
            lv, rv = self.amplify(l, self.cfg["tail"]), self.amplify(r, self.cfg["tail"])
            tails.setdefault(comp[0], (self.accumulate(lv), self.accumulate(rv)))

        def inter(a, b):
            return len(set(a) & set(b))

        edges = []
        keys = sorted(tails)
        for a in keys:
            for b in keys:
                if a < b:
                    (l1, r1), (l2, r2) = tails[a], tails[b]
                    s = max(inter(l1, l2), inter(l1, r2), inter(r1, l2), inter(r1, r2))
                    edges.append((a, b, s, self.good(a, b)))
        return [e for e in sort_conns(edges) if e[2] > 0]

    def to_string(self, cid):   # ReadComponent::to_string, ReadClusteringEngine.h:52-112
        reads = self.comps[cid]["reads"]
        counts = {0: 0, 1: 0}
        ends = {}
        for r in reads:
            c = self.cat[r]
            counts[c] = counts.get(c, 0) + 1
            ends.setdefault(c, []).extend([(self.start[r], True), (self.end[r], False)])
        parts = []
        for c in sorted(ends):
            cur, opened, iv = 0, 0, []
            for pos, is_start in sorted(ends[c]):   # (pos, False) before (pos, True)
                if is_start:
                    opened += 1
                    if opened == 1:
                        cur = pos
                else:
                    opened -= 1
                    if opened == 0:
                        iv.append(f"({cur},{pos})")
            parts.append(";".join(iv))
        return f"#{cid} : {'/'.join(str(counts[c]) for c in sorted(counts))} [{' / '.join(parts)}]"

    def print_components(self, ids):   # :189-198, sorts ids in place (largest first; ties by id here)
        if not self.debug:
            return
        ids.sort(key=lambda i: (-len(self.comps[i]["reads"]), i))
        self.printed.append(f"### Printing {len(ids)} components ###")
        self.printed += [self.to_string(i) for i in ids]
        self.printed.append("### ###")

    def run(self):   # :737-801
        c = self.cfg
        all_ids = sorted(self.comps)
        if c["sc_score"] > 0:
            ids = [i for i in all_ids if len(self.comps[i]["kmers"]) >= c["sc_score"]]
            conns = self.get_connections(ids, c["sc_score"])
            scaffold = [x for x in conns if x[2] > c["sc_score"]]
        else:
            conns = self.get_connections(all_ids, 1)
            scaffold = conns[:int(len(conns) * c["sc_fraction"])]
        cts = union_find(scaffold, set(), c["sc_min"], c["sc_max"])
        sids = self.merge([x[0] for x in cts])
        self.print_components(sids)
        if len(sids) > 2:
            strong = [x for x in self.core_connections(cts) if x[2] > 5]
            if strong:
                self.merge(spectral_clustering(strong, c["dims"]))
            self.remove_merged()
        core = self.ids(c["sc_min"])
        self.print_components(core)
        conns = self.get_connections(core, c["enrich"])
        cts = union_find(conns, set(core), 2, -1)
        self.merge([x[0] for x in cts])
        self.remove_merged()
        core = self.ids(c["sc_min"])
        self.print_components(core)
        return core
