"""Device-resident block batches (torch tensors in HBM) over the C ABI.

Used by bench.py and the GPU tests: upload a ``corpus.Corpus`` once, then
encode/decode it any number of times without host traffic.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass

import numpy as np
import torch

from . import snappy
from .corpus import Corpus


def _bound(lens: np.ndarray) -> np.ndarray:
    return 32 + lens.astype(np.uint64) + lens.astype(np.uint64) // 6


@dataclass
class Slots:
    """n variable-length slots in one device buffer."""
    buf: torch.Tensor      # uint8
    off: torch.Tensor      # int64
    len: torch.Tensor      # int32 (used length)
    cap: torch.Tensor      # int32 (capacity)
    max_cap: int

    @property
    def n(self) -> int:
        return int(self.off.numel())


def _spaced(caps: np.ndarray, device, align: int = 16) -> Slots:
    caps = caps.astype(np.uint64)
    stride = (caps + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    off = np.zeros(len(caps), dtype=np.uint64)
    if len(caps):
        off[1:] = np.cumsum(stride[:-1])
    total = int(stride.sum()) + 64
    return Slots(torch.empty(total, dtype=torch.uint8, device=device),
                 torch.from_numpy(off.astype(np.int64)).to(device),
                 torch.zeros(len(caps), dtype=torch.int32, device=device),
                 torch.from_numpy(caps.astype(np.int32)).to(device),
                 int(caps.max()) if len(caps) else 0)


def upload(c: Corpus, device="cuda") -> Slots:
    """Copy a corpus to the device, keeping its offsets."""
    buf = torch.from_numpy(np.ascontiguousarray(c.buf)).to(device)
    ln = c.len.astype(np.int32)
    return Slots(buf, torch.from_numpy(c.off.astype(np.int64)).to(device),
                 torch.from_numpy(ln).to(device), torch.from_numpy(ln).to(device),
                 int(ln.max()) if len(ln) else 0)


def encode_slots(raw: Slots) -> Slots:
    """Output slots spaced by the encode bound of each raw block."""
    lens = raw.len.cpu().numpy()
    return _spaced(_bound(lens), raw.buf.device)


def decode_slots(raw_lens: np.ndarray, device="cuda") -> Slots:
    return _spaced(raw_lens.astype(np.uint64), device)


def encode(raw: Slots, comp: Slots, stream=None) -> None:
    snappy.encode_batch(raw.buf, raw.off, raw.len, comp.buf, comp.off, comp.len, raw.max_cap,
                        stream)


def decode(comp: Slots, out: Slots, status: torch.Tensor, stream=None) -> None:
    snappy.decode_batch(comp.buf, comp.off, comp.len, out.buf, out.off, out.cap, out.len,
                        status, out.max_cap, stream)


def to_host(s: Slots) -> Corpus:
    return Corpus(s.buf.cpu().numpy(), s.off.cpu().numpy().astype(np.uint64),
                  s.len.cpu().numpy().astype(np.uint32))


def digest(s: Slots) -> tuple[str, int]:
    """SHA-256 of the concatenated used bytes of every slot, and their total."""
    c = to_host(s)
    h = hashlib.sha256()
    for i in range(c.n):
        o = int(c.off[i])
        h.update(memoryview(c.buf[o:o + int(c.len[i])]))
    return h.hexdigest(), c.raw_bytes
