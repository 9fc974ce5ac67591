"""On-disk container for coded video: a self-describing file of I-frame and
P-frame records with GOP / view muxing and a trailing index for random access to any GOP.

The reference has no container: its DVC path only estimates bits (DVC/net.py:57 calrealbits),
RLVC keeps compressai strings in memory (entropy_models.py:80-94) and I-frames go through BPG
files it deletes (models.py:412-429). Layout (little-endian):

  file    = "FVC1" | u16 version | u32 header_len | header (UTF-8 JSON) | record* | index
  record  = u8 kind ('I' | 'P') | u16 view | u32 gop | u16 frame | u32 payload_len | payload
  I payload = u16 h | u16 w | u8 levels | u16 q | u32 n_block_idx | block_idx (u8)
              | streams(coefficients)
  P payload = u8 precision (0 x3, 1 f32) | u8 framing (0 channel, 1 item, 2 segment)
              | u16 H/16 | u16 W/16 | u16 H/64 | u16 W/64 | streams(mv) | streams(z) | streams(feature)
  streams = u32 n | u32 len[n] (bytes) | bytes        (each stream byte-identical to compressai's
                                                      RansEncoder.encode_with_indexes output)
  index   = u32 n_records | (u8 kind, u16 view, u32 gop, u16 frame, u64 offset)* | u64 index_offset | "FVCX"

The header carries the codec name / level, frame geometry, GOP length, view and GOP counts, the
I-frame transform parameters and a CRC-32 of every entropy table, which a reader checks against
its own model before decoding.
"""
from __future__ import annotations

import io
import json
import struct
import zlib

import numpy as np
import torch

from . import iframe as IF
from .entropy_models import EncodedStreams
from .net import FRAMINGS, PFrameBitstream

MAGIC = b"FVC1"
INDEX_MAGIC = b"FVCX"
VERSION = 1
_REC = struct.Struct("<cHIHI")
_IDX = struct.Struct("<cHIHQ")


def tables_crc(model) -> str:
    """CRC-32 over the model's quantised CDF tables (mv, z, feature) and scale table."""
    model.update()
    return tables_crc_of(*model._coders["tables"])


def tables_crc_of(tz, tmv, tf) -> str:
    """tables_crc of host tables (FactorizedTables z / mv, LaplaceTables feature)."""
    c = 0
    for t in (tmv, tz, tf):
        for a in (t.cdf, t.cdf_length, t.offset):
            c = zlib.crc32(np.ascontiguousarray(a, np.int32).tobytes(), c)
    c = zlib.crc32(np.ascontiguousarray(tf.scale_table, np.float32).tobytes(), c)
    return f"{c:08x}"


def _pack_streams(strings) -> bytes:
    return struct.pack(f"<I{len(strings)}I", len(strings), *[len(s) for s in strings]) + b"".join(strings)


def _unpack_streams(buf, pos):
    (n,) = struct.unpack_from("<I", buf, pos)
    pos += 4
    lens = struct.unpack_from(f"<{n}I", buf, pos)
    pos += 4 * n
    out = []
    for L in lens:
        out.append(bytes(buf[pos:pos + L]))
        pos += L
    return out, pos


def split_pframes(bs: PFrameBitstream):
    """Per-frame payloads of a batched P-frame bitstream: [(mv, z, feature) stream lists]."""
    parts = {k: getattr(bs, k).to_bytes_list() for k in ("mv", "z", "feature")}
    out = []
    for b in range(bs.batch):
        fr = []
        for k in ("mv", "z", "feature"):
            s = parts[k]
            per = len(s) // bs.batch
            fr.append(s[b * per:(b + 1) * per])
        out.append(fr)
    return out


def pframe_payload(bs: PFrameBitstream, b: int = 0, frame_streams=None) -> bytes:
    fs = frame_streams if frame_streams is not None else split_pframes(bs)[b]
    (H16, W16), (H64, W64) = bs.hw16, bs.hw64
    head = struct.pack("<BBHHHH", 1 if bs.precision == "f32" else 0, FRAMINGS.index(bs.framing), H16, W16, H64, W64)
    return head + b"".join(_pack_streams(s) for s in fs)


def pframe_from_payload(payload: bytes, device) -> PFrameBitstream:
    prec, fr, H16, W16, H64, W64 = struct.unpack_from("<BBHHHH", payload, 0)
    pos = 10
    parts = []
    for _ in range(3):
        s, pos = _unpack_streams(payload, pos)
        parts.append(EncodedStreams.from_bytes_list(s, device))
    return PFrameBitstream(parts[0], parts[1], parts[2], 1, (H16, W16), (H64, W64), FRAMINGS[fr],
                           "f32" if prec else "x3")


def iframe_payload(bs: IF.IFrameBitstream) -> bytes:
    if bs.batch != 1:
        raise ValueError("one I-frame per record")
    bidx = np.ascontiguousarray(bs.block_index, np.uint8).tobytes()
    head = struct.pack("<HHBHI", bs.h, bs.w, bs.levels, bs.q, len(bidx))
    return head + bidx + _pack_streams(bs.streams.to_bytes_list())


def iframe_from_payload(payload: bytes, device) -> IF.IFrameBitstream:
    h, w, levels, q, nb = struct.unpack_from("<HHBHI", payload, 0)
    pos = struct.calcsize("<HHBHI")
    bidx = np.frombuffer(payload, np.uint8, nb, pos).reshape(3, h // IF.BLOCK, w // IF.BLOCK).copy()
    pos += nb
    strings, pos = _unpack_streams(payload, pos)
    return IF.IFrameBitstream(1, h, w, levels, q, bidx, EncodedStreams.from_bytes_list(strings, device))


class ContainerWriter:
    def __init__(self, f, header: dict):
        self.f = f
        self.index = []
        hb = json.dumps(header, sort_keys=True).encode()
        f.write(MAGIC + struct.pack("<HI", VERSION, len(hb)) + hb)

    def _record(self, kind, view, gop, frame, payload):
        self.index.append((kind, view, gop, frame, self.f.tell()))
        self.f.write(_REC.pack(kind, view, gop, frame, len(payload)))
        self.f.write(payload)

    def write_iframe(self, view, gop, frame, bs: IF.IFrameBitstream):
        self._record(b"I", view, gop, frame, iframe_payload(bs))

    def write_pframe(self, view, gop, frame, payload: bytes):
        self._record(b"P", view, gop, frame, payload)

    def close(self):
        pos = self.f.tell()
        self.f.write(struct.pack("<I", len(self.index)))
        for e in self.index:
            self.f.write(_IDX.pack(*e))
        self.f.write(struct.pack("<Q", pos) + INDEX_MAGIC)


class ContainerReader:
    def __init__(self, data: bytes):
        self.data = memoryview(data)
        if bytes(self.data[:4]) != MAGIC:
            raise ValueError("not an FVC1 container")
        ver, hl = struct.unpack_from("<HI", self.data, 4)
        if ver != VERSION:
            raise ValueError(f"unsupported container version {ver}")
        self.header = json.loads(bytes(self.data[10:10 + hl]).decode())
        if bytes(self.data[-4:]) != INDEX_MAGIC:
            raise ValueError("missing index")
        (ipos,) = struct.unpack_from("<Q", self.data, len(self.data) - 12)
        (n,) = struct.unpack_from("<I", self.data, ipos)
        self.index = [_IDX.unpack_from(self.data, ipos + 4 + i * _IDX.size) for i in range(n)]

    def record(self, entry):
        kind, view, gop, frame, off = entry
        k2, v2, g2, f2, L = _REC.unpack_from(self.data, off)
        if (k2, v2, g2, f2) != (kind, view, gop, frame):
            raise ValueError("index does not match record")
        start = off + _REC.size
        return bytes(self.data[start:start + L])

    def gop_records(self, view, gop):
        return sorted((e for e in self.index if e[1] == view and e[2] == gop), key=lambda e: e[3])

    def gops(self):
        return sorted({(e[1], e[2]) for e in self.index})


def encode_video(model, video: torch.Tensor, f, iframe_q=None, framing="segment", views=None):
    """Encode video [N, T, 3, H, W] (N GOPs, H and W multiples of 64) into container file f.
    GOP n is muxed as (view = views[n] if given else 0, gop = n). Frame 0 of each GOP is coded by
    the I-frame codec (step iframe_q, default from model.I_level: iframe.iframe_step), frames
    1..T-1 by the P-frame codec against the encoder's own previous reconstruction (what the
    decoder will hold). Returns the encoder's reconstructions [N, T, 3, H, W]."""
    N, T, C, H, W = video.shape
    q = IF.iframe_step(model.I_level) if iframe_q is None else int(iframe_q)
    header = {"codec": model.name, "level": model.compression_level, "height": H, "width": W, "gop": T,
              "gops": N, "tables_crc32": tables_crc(model), "framing": framing,
              "iframe": {"transform": "rct+legall53", "levels": IF.LEVELS, "block": IF.BLOCK,
                         "band_rows": IF.BAND_ROWS, "q": q}}
    w = ContainerWriter(f, header)
    recons = torch.empty_like(video)
    for n in range(N):
        v = 0 if views is None else int(views[n])
        ibs, x = IF.encode(video[n, 0:1].contiguous(), q)
        w.write_iframe(v, n, 0, ibs)
        recons[n, 0] = x[0]
        for t in range(1, T):
            bs, x = model.compress(video[n, t:t + 1].contiguous(), x, framing=framing)
            w.write_pframe(v, n, t, pframe_payload(bs))
            recons[n, t] = x[0]
    w.close()
    return recons


def decode_video(model, data: bytes, device=None):
    """Decode every GOP of a container: {(view, gop): frames [T, 3, H, W]} on the device."""
    r = ContainerReader(data)
    if r.header.get("tables_crc32") != tables_crc(model):
        raise ValueError("container was coded with different entropy tables (model weights differ)")
    dev = torch.device(device) if device is not None else next(model.parameters()).device
    out = {}
    for view, gop in r.gops():
        frames = []
        x = None
        for e in r.gop_records(view, gop):
            payload = r.record(e)
            if e[0] == b"I":
                x = IF.decode(iframe_from_payload(payload, dev))
            else:
                x = model.decompress(pframe_from_payload(payload, dev), x)
            frames.append(x[0])
        out[(view, gop)] = torch.stack(frames)
    return out


def encode_video_bytes(model, video, **kw):
    buf = io.BytesIO()
    rec = encode_video(model, video, buf, **kw)
    return buf.getvalue(), rec
