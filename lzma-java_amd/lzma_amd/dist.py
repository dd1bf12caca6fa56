"""Multi-GPU output gather and the multi-member container.

Each rank encodes its own independent streams (no data-path collective). After
that, ONE exchange collects every rank's packed payloads on one rank:

  1. all_gather of the per-rank stream counts, then of the per-stream
     compressed sizes (8 B per stream);
  2. point-to-point send/recv of each rank's packed payload into the
     destination's contiguous buffer (RCCL over xGMI with backend "nccl",
     gloo on CPU tensors in the tests).

An .lzma file holds exactly one stream (LzmaAlone.java:208-218), so the
gathered output is written as a multi-member container (`pack_container`).
Every member is a standard .lzma file (13-byte header + payload) that the
reference Decoder reads unchanged.
"""
from __future__ import annotations

import struct
from typing import List, Optional, Sequence, Tuple

import numpy as np

MAGIC = b"LZMG"
VERSION = 1


def gather_streams(payload, lens: np.ndarray, dst: int = 0, group=None) -> Tuple[Optional[object], Optional[np.ndarray], Optional[np.ndarray]]:
    """Collect every rank's packed payload on rank `dst`.

    payload: 1-D uint8 torch tensor holding this rank's streams back to back
             (at least sum(lens) bytes); lens: compressed size per stream.
    Returns on dst: (gathered uint8 tensor, all lens in rank order, per-rank
    stream counts); on other ranks: (None, None, None).
    """
    import torch
    import torch.distributed as td

    world = td.get_world_size(group)
    rank = td.get_rank(group)
    dev = payload.device
    lens = np.asarray(lens, dtype=np.int64)
    cnt = torch.tensor([lens.size], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    td.all_gather(cnts, cnt, group=group)
    counts = np.array([int(c.item()) for c in cnts], dtype=np.int64)
    mx = int(counts.max()) if world else 0
    mine = torch.zeros(max(mx, 1), dtype=torch.int64, device=dev)
    if lens.size:
        mine[:lens.size] = torch.from_numpy(lens).to(dev)
    all_l = [torch.zeros_like(mine) for _ in range(world)]
    td.all_gather(all_l, mine, group=group)
    per_rank = [all_l[r][:counts[r]].cpu().numpy() for r in range(world)]
    nbytes = [int(x.sum()) for x in per_rank]
    if rank == dst:
        out = torch.empty(sum(nbytes), dtype=torch.uint8, device=dev)
        offs = np.concatenate([[0], np.cumsum(nbytes)]).astype(np.int64)
        reqs = []
        for r in range(world):
            if nbytes[r] == 0:
                continue
            view = out[int(offs[r]):int(offs[r + 1])]
            if r == rank:
                view.copy_(payload[:nbytes[r]])
            else:
                reqs.append(td.irecv(view, src=_global(r, group), group=group))
        for q in reqs:
            q.wait()
        return out, np.concatenate(per_rank) if per_rank else np.zeros(0, np.int64), counts
    if nbytes[rank]:
        td.send(payload[:nbytes[rank]].contiguous(), dst=_global(dst, group), group=group)
    return None, None, None


def rank_streams(nstreams: int, rank: int, world: int) -> np.ndarray:
    """Streams of `rank` when one buffer's independent streams are dealt round-robin
    over `world` ranks (rank r takes {i : i mod G = r})."""
    return np.arange(rank, nstreams, world, dtype=np.int64)


def stream_order(counts: Sequence[int], world: int) -> np.ndarray:
    """Global stream index of every gathered stream, for payloads gathered in rank
    order (rank 0's streams, then rank 1's, ...) from a round-robin deal."""
    idx = [rank_streams(int(sum(counts)), r, world)[:int(counts[r])] for r in range(world)]
    return np.concatenate(idx) if idx else np.zeros(0, np.int64)


def reorder_payloads(gathered: bytes, lens: Sequence[int], order: Sequence[int]) -> List[bytes]:
    """Split a gathered buffer into its streams and put them back in global order."""
    offs = np.concatenate([[0], np.cumsum(np.asarray(lens, dtype=np.int64))])
    out: List[bytes] = [b""] * len(order)
    for k, g in enumerate(order):
        out[int(g)] = gathered[int(offs[k]):int(offs[k + 1])]
    return out


def _global(r: int, group) -> int:
    import torch.distributed as td
    if group is None:
        return r
    return td.get_global_rank(group, r)


def pack_container(props: bytes, payloads: Sequence[bytes], sizes: Sequence[int]) -> bytes:
    """Multi-member container: b"LZMG" | u32 version | u64 count |
    count x (u64 offset, u64 length) | members, each a standard .lzma file
    (5 props + u64 size + payload, LzmaAlone.java:208-217)."""
    if len(props) != 5:
        raise ValueError("props must be 5 bytes")
    if len(payloads) != len(sizes):
        raise ValueError("payloads and sizes differ in length")
    head = len(MAGIC) + 4 + 8 + 16 * len(payloads)
    table, members, off = [], [], head
    for pl, n in zip(payloads, sizes):
        m = props + (int(n) & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little") + bytes(pl)
        table.append(struct.pack("<QQ", off, len(m)))
        members.append(m)
        off += len(m)
    return MAGIC + struct.pack("<IQ", VERSION, len(payloads)) + b"".join(table) + b"".join(members)


def unpack_container(blob: bytes) -> List[bytes]:
    """Members (.lzma files) of a pack_container blob; raises ValueError if malformed."""
    if len(blob) < 16 or blob[:4] != MAGIC:
        raise ValueError("not an LZMG container")
    ver, n = struct.unpack_from("<IQ", blob, 4)
    if ver != VERSION:
        raise ValueError("unsupported container version %d" % ver)
    if 16 + 16 * n > len(blob):
        raise ValueError("truncated member table")
    out = []
    for i in range(n):
        off, ln = struct.unpack_from("<QQ", blob, 16 + 16 * i)
        if off + ln > len(blob) or ln < 13:
            raise ValueError("member %d out of range" % i)
        out.append(blob[off:off + ln])
    return out
