"""Ingest re-partition for N GPUs.

Synthetic runs generate each rank's packets already partitioned by flow group
(cilium_amd/stream.py pair_rank).  Real traffic arrives on whatever rank the
NIC's RSS picked, so before classification each rank computes the owner of
every frame — the rank of its flow group, the unordered address pair
handle_policy's conntrack sees after bpf_lb's translation
(gf_pipeline_partition, a HIP kernel) — and the frames move to their owners in
one all-to-all (RCCL over xGMI on GPUs, gloo in the CPU tests).  A rank's
batch is then the concatenation of what it received in source-rank order, so
every flow group is classified by one rank, in (source rank, arrival) order.
"""
import ctypes as C

import numpy as np

from ._lib import lib, gf_frames, gf_pipe_batch


def partition(dp, frames, lens, rank, world, flow_hash=None, tc_index=None):
    """Owner rank, stable owner order and per-rank counts of a frame batch
    (device tensors), through the pipeline program's bpf_lb tables."""
    import torch
    from .datapath import _check, _ptr, _stream
    n = frames.shape[0]
    dev = frames.device
    owner = torch.empty(n, dtype=torch.int32, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.empty(world, dtype=torch.int32, device=dev)
    pb = gf_pipe_batch(gf_frames(n, frames.shape[1] if n else 64, _ptr(frames), _ptr(lens)), _ptr(tc_index),
                       _ptr(flow_hash))
    _check(lib.gf_pipeline_partition(dp.pipe, C.byref(pb), rank, world, _ptr(owner), _ptr(order), _ptr(counts),
                                     _stream()), "gf_pipeline_partition")
    return owner, order, counts


def exchange(order, counts, tensors, group=None):
    """All-to-all of per-packet tensors (first dimension = packet): packets go
    to their owner in `order`, `counts[r]` of them to rank r.  Returns the
    received tensors, source rank 0's packets first."""
    import torch
    import torch.distributed as dist
    counts = counts.to(torch.int64)
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    send_splits = counts.cpu().tolist()
    recv_splits = recv_counts.cpu().tolist()
    total = int(sum(recv_splits))
    order = order.to(torch.int64)
    out = []
    for t in tensors:
        if t is None:
            out.append(None)
            continue
        signed = {torch.uint32: torch.int32, torch.uint16: torch.int16, torch.uint64: torch.int64}.get(t.dtype)
        src = t.view(signed) if signed is not None else t          # index_select has no unsigned wide types
        send = src.index_select(0, order).contiguous()
        recv = torch.empty((total,) + tuple(t.shape[1:]), dtype=src.dtype, device=t.device)
        dist.all_to_all_single(recv, send, recv_splits, send_splits, group=group)
        out.append(recv.view(t.dtype) if signed is not None else recv)
    return out


# ---- host restatement of the owner rule (test checker) ----
def _hash_words(w, nbytes):
    """gf_hash_words (csrc/gf_common.h) over uint32 rows [n, k]."""
    m = np.uint32
    h = np.full(w.shape[0], 0x9747b28c ^ nbytes, np.uint32)
    rotl = lambda x, r: ((x << m(r)) | (x >> m(32 - r))).astype(np.uint32)
    with np.errstate(over="ignore"):
        for j in range(w.shape[1]):
            k = (w[:, j].astype(np.uint32) * m(0xcc9e2d51)).astype(np.uint32)
            k = rotl(k, 15)
            k = (k * m(0x1b873593)).astype(np.uint32)
            h ^= k
            h = rotl(h, 13)
            h = (h * m(5) + m(0xe6546b64)).astype(np.uint32)
        h ^= h >> m(16); h = (h * m(0x85ebca6b)).astype(np.uint32)
        h ^= h >> m(13); h = (h * m(0xc2b2ae35)).astype(np.uint32)
        h ^= h >> m(16)
    return h


def pair_rank6(s6, d6, world):
    """gf_pair_hash6 (big-endian lexicographic order of the two addresses) mod world."""
    s6, d6 = np.asarray(s6, np.uint8), np.asarray(d6, np.uint8)
    less = np.array([bytes(a) < bytes(b) for a, b in zip(s6, d6)], bool)
    lo = np.where(less[:, None], s6, d6)
    hi = np.where(less[:, None], d6, s6)
    w = np.concatenate([lo, hi], axis=1).copy().view("<u4")
    return (_hash_words(w, 32) % np.uint32(world)).astype(np.int64)
