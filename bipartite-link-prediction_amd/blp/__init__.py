"""blp — MI355X-native bipartite link-scoring engine (host side).

The compute lives in ``libblp.so`` (HIP kernels for gfx950, C-ABI in include/blp.h).
This package binds it with ctypes and keeps the data contract of the reference's
scripts; the reference-named modules (similarity, svd, random_walks, util, eval,
dataset_maker) one directory up are the drop-in call surface.
"""
from ._lib import ADAMIC, CN, JACCARD, BLPError, BLPUnavailable, device_count, device_sync, lib, prewarm, version
from .topk import TopK
from .graph import DeviceGraph, HostGraph, LoadEdgeList, PairBatch, load_edge_list, parse_edge_list

__all__ = [
    "ADAMIC", "CN", "JACCARD", "BLPError", "BLPUnavailable", "DeviceGraph", "HostGraph", "LoadEdgeList",
    "PairBatch", "TopK", "device_count", "device_sync", "lib", "load_edge_list", "parse_edge_list", "prewarm", "version",
]
