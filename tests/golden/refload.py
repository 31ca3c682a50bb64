"""In-memory loader for the reference's Python-2 scripts (fixture generation only).

THIS FILE IS TEST INFRASTRUCTURE. It is only ever run in the build container, where
``/root/reference`` exists, by ``tests/golden/make_golden.py``. It never travels to
the GPU box in any useful form (nothing under ``tests/`` or the product imports it at
run time), and it contains no reference source: it reads the reference files as text,
translates them with the stdlib ``lib2to3`` and ``exec``s them into fresh module
objects ("Working oracle").

Two shims stand in for what the reference imports but the image lacks:

* ``sets``  -> ``Set = set`` (``similarity.py:5``).
* ``snap``  -> a tiny pure-Python undirected graph that follows SNAP's *documented*
  ``TUNGraph`` semantics for the calls the reference makes
  (``similarity.py:16,22,29,41,74,85,121``; ``dataset_maker.py:84,97,101,139``):
  ``LoadEdgeList`` (whitespace columns, ``#`` comment lines skipped, multi-edges
  deduplicated, a self-loop stored once in the node's own neighbour vector so that
  ``GetDeg`` counts it once), ``GetNodesAtHop`` (nodes at *exact* BFS distance h) and
  ``GetNI(n).GetDeg()``. SNAP itself is absent (``.MISSING_LARGE_BLOBS:1-3``), so this
  boundary is "parity unpinned" (SURVEY.md §8(c)); it is cross-checked against an
  independent scipy formulation in ``tests/test_oracle.py``.
"""
import os
import sys
import types
from collections import deque

REF = os.environ.get("BLP_REFERENCE_DIR", "/root/reference")


# --------------------------------------------------------------------------- snap shim
class _NI:
    def __init__(self, g, n):
        self._g, self._n = g, n

    def GetId(self):
        return self._n

    def GetDeg(self):
        return len(self._g._adj[self._n])

    def GetOutDeg(self):
        return len(self._g._adj[self._n])


class _TUNGraph:
    def __init__(self):
        self._adj = {}

    def AddNode(self, n):
        self._adj.setdefault(n, set())

    def AddEdge(self, a, b):
        self.AddNode(a)
        self.AddNode(b)
        self._adj[a].add(b)
        self._adj[b].add(a)  # a == b: stored once (SNAP TUNGraph::AddEdge)

    def Nodes(self):
        for n in self._adj:
            yield _NI(self, n)

    def GetNI(self, n):
        return _NI(self, n)

    def GetNodes(self):
        return len(self._adj)

    def GetEdges(self):
        loops = sum(1 for n, s in self._adj.items() if n in s)
        return (sum(len(s) for s in self._adj.values()) - loops) // 2 + loops

    def IsNode(self, n):
        return n in self._adj


def _make_snap():
    m = types.ModuleType("snap")
    m.PUNGraph = _TUNGraph
    m.TIntV = list

    def LoadEdgeList(kind, path, c0=0, c1=1):
        g = _TUNGraph()
        with open(path) as f:
            for line in f:
                if line.startswith("#"):
                    continue
                cols = line.split()
                if len(cols) <= max(c0, c1):
                    continue
                g.AddEdge(int(cols[c0]), int(cols[c1]))
        return g

    def Nodes(g):
        return g.Nodes()

    def GetNodesAtHop(g, start, hop, vec, is_dir=False):
        dist = {start: 0}
        q = deque([start])
        while q:
            n = q.popleft()
            if dist[n] == hop:
                continue
            for w in sorted(g._adj[n]):
                if w not in dist:
                    dist[w] = dist[n] + 1
                    q.append(w)
        del vec[:]
        vec.extend(n for n, d in dist.items() if d == hop)
        return len(vec)

    m.LoadEdgeList = LoadEdgeList
    m.Nodes = Nodes
    m.GetNodesAtHop = GetNodesAtHop
    return m


def _make_sets():
    m = types.ModuleType("sets")
    m.Set = set
    return m


# --------------------------------------------------------------------------- loader
def _translate(src):
    from lib2to3 import refactor

    tool = refactor.RefactoringTool(refactor.get_fixers_from_package("lib2to3.fixes"))
    return str(tool.refactor_string(src, "<ref>"))


def load(names=("util", "dataset_maker", "similarity", "svd", "eval", "random_walks")):
    """Translate and exec the named reference scripts; returns {name: module}."""
    import warnings

    warnings.filterwarnings("ignore")
    os.environ.setdefault("MPLBACKEND", "Agg")
    import scipy.sparse.linalg  # noqa: F401  (svd.py:24 uses sparse.linalg.svds)
    import networkx as nx
    import scipy.sparse as sp

    sys.modules["snap"] = _make_snap()
    sys.modules["sets"] = _make_sets()
    # random_walks.py:27 calls .getrow(), which scipy's csr_array dropped.
    if not getattr(nx, "_blp_wrapped", False):
        _orig = nx.adjacency_matrix

        def adjacency_matrix(G, *a, **k):
            return sp.csr_matrix(_orig(G, *a, **k))

        nx.adjacency_matrix = adjacency_matrix
        nx._blp_wrapped = True
    mods = {}
    for name in names:
        path = os.path.join(REF, name + ".py")
        with open(path) as f:
            src = f.read()
        code = _translate(src.expandtabs(8))  # Python 2 tab semantics
        mod = types.ModuleType(name)
        mod.__file__ = "<reference:%s.py>" % name
        sys.modules[name] = mod
        exec(compile(code, mod.__file__, "exec"), mod.__dict__)
        mods[name] = mod
    return mods
