"""Zero-copy NPZ reader for the client-update wire format.

Clients write their weights with NpzWeightsSerializer (serialization.py:280-306,
`np.savez`, ZIP_STORED unless compress_model is set; client.py:186-199).  An
uncompressed .npz is a zip whose members arr_0.npy, arr_1.npy, ... hold raw
.npy payloads, so every layer can be viewed in place inside the blob:

    local file header (30 B + name + extra) -> .npy magic/header -> raw data

`npz_views(blob)` returns numpy views into `blob` (no copy), in member order —
the same order as `list(np.load(f).values())` — so the ingest pipeline can
memcpy each layer straight into a pinned staging row.  Compressed members,
Fortran-ordered or object arrays, and anything unexpected fall back to
np.load (allow_pickle=False), so results never depend on which path ran.
"""
from __future__ import annotations

import ast
import io
import struct
import zipfile
from typing import List, Optional

import numpy as np

_LOCAL_HDR = struct.Struct("<IHHHHHIIIHH")  # zip local file header (30 bytes)
_LOCAL_SIG = 0x04034B50


def _npy_payload(buf: memoryview, off: int):
    """Parse a .npy header at `off`; return (dtype, shape, data_offset) or None."""
    if bytes(buf[off:off + 6]) != b"\x93NUMPY":
        return None
    major = buf[off + 6]
    if major == 1:
        hlen = struct.unpack_from("<H", buf, off + 8)[0]
        hstart = off + 10
    elif major in (2, 3):
        hlen = struct.unpack_from("<I", buf, off + 8)[0]
        hstart = off + 12
    else:
        return None
    try:
        hdr = ast.literal_eval(bytes(buf[hstart:hstart + hlen]).decode("latin1"))
    except (ValueError, SyntaxError):
        return None
    if not isinstance(hdr, dict) or hdr.get("fortran_order"):
        return None
    dt = np.dtype(hdr["descr"])
    if dt.hasobject:
        return None
    return dt, tuple(hdr["shape"]), hstart + hlen


class _ViewFile(io.RawIOBase):
    """Minimal read-only seekable file over a memoryview (zipfile reads only
    the central directory through it)."""

    def __init__(self, mv: memoryview):
        self.mv, self.pos = mv.cast("B"), 0

    def readable(self):
        return True

    def seekable(self):
        return True

    def tell(self):
        return self.pos

    def seek(self, off, whence=0):
        self.pos = off if whence == 0 else (self.pos + off if whence == 1 else len(self.mv) + off)
        return self.pos

    def readinto(self, b):
        n = max(0, min(len(b), len(self.mv) - self.pos))
        b[:n] = self.mv[self.pos:self.pos + n]
        self.pos += n
        return n


def npz_views(blob) -> Optional[List[np.ndarray]]:
    """Layer views into an uncompressed NPZ blob, or None if it needs np.load."""
    buf = memoryview(blob)
    # BytesIO shares a bytes object's buffer (no copy); anything else is
    # wrapped read-only without copying the payload via a file-like view.
    src = io.BytesIO(blob) if isinstance(blob, bytes) else _ViewFile(buf)
    try:
        with zipfile.ZipFile(src) as zf:
            infos = zf.infolist()
    except zipfile.BadZipFile:
        return None
    out = []
    for info in infos:
        if info.compress_type != zipfile.ZIP_STORED or not info.filename.endswith(".npy"):
            return None
        off = info.header_offset
        fields = _LOCAL_HDR.unpack_from(buf, off)
        if fields[0] != _LOCAL_SIG:
            return None
        name_len, extra_len = fields[9], fields[10]
        data = off + _LOCAL_HDR.size + name_len + extra_len
        parsed = _npy_payload(buf, data)
        if parsed is None:
            return None
        dt, shape, start = parsed
        count = int(np.prod(shape)) if shape else 1
        if start + count * dt.itemsize > data + info.file_size:
            return None
        out.append(np.frombuffer(buf, dtype=dt, count=count, offset=start).reshape(shape))
    return out


_CODE_TO_DTYPE = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.int64, 5: np.float16, 6: np.uint8,
                  7: np.int8, 8: np.bool_}
MAX_LAYERS = 4096


def native_views(blob) -> Optional[List[np.ndarray]]:
    """Same as npz_views, with the member index built by fa_npz_index (C++)."""
    import ctypes
    from . import _lib
    L = _lib.load()
    buf = memoryview(blob).cast("B")
    n = len(buf)
    if n == 0:
        return None
    src = np.frombuffer(buf, dtype=np.uint8)
    offs = np.empty(MAX_LAYERS, np.int64)
    cnts = np.empty(MAX_LAYERS, np.int64)
    dts = np.empty(MAX_LAYERS, np.int32)
    nds = np.empty(MAX_LAYERS, np.int32)
    shp = np.empty(MAX_LAYERS * 8, np.int64)
    k = L.fa_npz_index(src.ctypes.data_as(ctypes.c_void_p), n, offs.ctypes.data, cnts.ctypes.data,
                       dts.ctypes.data, nds.ctypes.data, shp.ctypes.data, MAX_LAYERS)
    if k < 0:
        return None
    out = []
    for i in range(k):
        dt = np.dtype(_CODE_TO_DTYPE[int(dts[i])])
        shape = tuple(int(x) for x in shp[i * 8: i * 8 + int(nds[i])])
        out.append(np.frombuffer(buf, dtype=dt, count=int(cnts[i]), offset=int(offs[i])).reshape(shape))
    return out


def read_layers(blob) -> List[np.ndarray]:
    """Layers of an NPZ blob: zero-copy views (native index) when possible, np.load otherwise."""
    v = native_views(blob)
    if v is not None:
        return v
    with io.BytesIO(bytes(blob)) as f:
        with np.load(f, allow_pickle=False) as z:
            return [z[k] for k in z.files]


# ---------------------------------------------------------------------------
# writer: byte-identical np.savez(BytesIO, *arrays) for the saved global model
# ---------------------------------------------------------------------------
def write_npz(arrays) -> Optional[bytes]:
    """`np.savez` of `arrays` into memory, byte for byte, with the member
    checksums computed natively (fa_crc32, threaded) and each payload copied
    once.

    np.savez (numpy `_savez`) opens member arr_i.npy with
    `zipfile.ZipFile.open(name, 'w', force_zip64=True)` on a ZIP_STORED,
    allowZip64 archive and streams the .npy header and the raw C-order data
    through it; zipfile checksums every write with zlib.crc32 and rewrites the
    local header at the end.  Here the same ZipInfo fields are filled in
    directly and written once, and zipfile itself writes the central
    directory, so the archive layout is zipfile's own.  The reference saves
    the aggregated model this way (NpzWeightsSerializer.serialize,
    serialization.py:290-296 -> ParameterDao.save, aggregation.py:139-147).

    Returns None (the caller runs np.savez) for anything numpy writes another
    way: object dtypes (pickled), arrays that are not C-contiguous, members of
    4 GiB or more; and when libfedavg_hip.so cannot be loaded.
    """
    from numpy.lib import format as npformat
    from . import _lib

    arrs = [np.asanyarray(a) for a in arrays]
    for a in arrs:
        if a.dtype.hasobject or not a.flags.c_contiguous or a.nbytes >= zipfile.ZIP64_LIMIT:
            return None
    try:
        # host-only helpers of the HIP library (CRC-32, threaded copies); a
        # process that only saves a model must still save it without them
        L = _lib.load()
    except (_lib.AggregationError, OSError):
        return None  # the caller runs np.savez: the same bytes
    import ctypes
    crc = ctypes.c_uint32()
    parts: list = []  # local header, .npy header, payload for each member; then the directory
    infos = []
    offset = 0
    for i, a in enumerate(arrs):
        hdr = io.BytesIO()
        npformat._write_array_header(hdr, npformat.header_data_from_array_1_0(a), None)
        hdr = hdr.getvalue()
        data = a.reshape(-1).view(np.uint8) if a.nbytes else np.empty(0, np.uint8)
        zi = zipfile.ZipInfo("arr_%d.npy" % i)  # as ZipFile.open(name, 'w'): default date_time
        zi.compress_type = zipfile.ZIP_STORED
        zi._compresslevel = None
        zi.flag_bits = 0x00  # seekable output: no data descriptor
        zi.external_attr = 0o600 << 16
        zi.file_size = zi.compress_size = len(hdr) + data.nbytes
        _lib.check(L.fa_crc32(data.ctypes.data if data.nbytes else None, data.nbytes,
                              zlib_crc32(hdr), 0, ctypes.byref(crc)), "fa_crc32")
        zi.CRC = crc.value
        zi.header_offset = offset
        lh = zi.FileHeader(True)  # force_zip64=True, as np.savez
        parts += [lh, hdr, data.data]
        infos.append(zi)
        offset += len(lh) + len(hdr) + data.nbytes
    # zipfile writes the central directory and end records itself, to a
    # stream that reports the archive offsets
    tail = _OffsetStream(offset)
    zf = zipfile.ZipFile(tail, mode="w", compression=zipfile.ZIP_STORED, allowZip64=True)
    for zi in infos:
        zf.filelist.append(zi)
        zf.NameToInfo[zi.filename] = zi
    zf._didModify = True
    zf.close()
    parts.append(tail.getvalue())
    from .engine import _hostfast
    if _hostfast is None:
        return b"".join(parts)  # one allocation, each part copied once
    # one allocation, every part copied once by the threaded fa_pack (the GIL
    # released) into the new bytes object before anyone else sees it
    bufs = [np.frombuffer(p_, dtype=np.uint8) for p_ in parts]
    sizes = np.fromiter((b.nbytes for b in bufs), dtype=np.int64, count=len(bufs))
    offs = np.zeros(len(bufs), dtype=np.int64)
    np.cumsum(sizes[:-1], out=offs[1:])
    total = int(sizes.sum())
    out, addr = _hostfast.alloc_bytes(total)
    srcs = np.fromiter((b.ctypes.data if b.nbytes else 0 for b in bufs), dtype=np.uint64, count=len(bufs))
    _lib.check(L.fa_pack(addr, offs.ctypes.data, srcs.ctypes.data, sizes.ctypes.data, len(bufs), 0), "fa_pack")
    return out


class _OffsetStream(io.RawIOBase):
    """Writable, seekable stream whose positions start at `base` (the bytes
    before it are the members, assembled separately)."""

    def __init__(self, base: int):
        super().__init__()
        self.base = base
        self.inner = io.BytesIO()

    def writable(self):
        return True

    def seekable(self):
        return True

    def write(self, b):
        return self.inner.write(b)

    def tell(self):
        return self.base + self.inner.tell()

    def seek(self, pos, whence=io.SEEK_SET):
        if whence == io.SEEK_SET:
            if pos < self.base:
                raise ValueError("seek before the directory")
            return self.base + self.inner.seek(pos - self.base)
        return self.base + self.inner.seek(pos, whence)

    def getvalue(self):
        return self.inner.getvalue()


def zlib_crc32(b: bytes) -> int:
    import zlib
    return zlib.crc32(b)
