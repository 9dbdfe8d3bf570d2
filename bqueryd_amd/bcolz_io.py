"""bcolz on-disk layout: reader and writer (host side; blosc via libblosc).

bqueryd's shards (``*.bcolz`` / ``*.bcolzs``, ``bqueryd/worker.py:32-33``) and its per-shard
results (``worker.py:335-346``: ``result_ctable.flush()`` then a tar of the rootdir) are bcolz
ctable directories.  bcolz is not vendored in the reference, so the layout below
is restated from the public bcolz 1.x design [ext-bcolz, unverified]:

  <ctable>/__rootdirs__    JSON {"names": [...], "dirs": {name: name}}
  <ctable>/__attrs__       JSON {}
  <ctable>/<col>/__attrs__ JSON {}
  <ctable>/<col>/meta/sizes    JSON {"shape": [n], "nbytes": n*itemsize, "cbytes": c}
  <ctable>/<col>/meta/storage  JSON {"dtype", "cparams": {clevel, shuffle, cname, quantize},
                                     "chunklen", "expectedlen", "dflt"}
  <ctable>/<col>/data/__<i>.blp  16-byte bloscpack header ('blpk', version, 3 reserved bytes,
                                  int64 nchunks=1) + one blosc1 frame; chunks hold `chunklen`
                                  items, the last ("leftover") chunk holds the remainder.

The blosc frames are produced/decoded by the system c-blosc 1.x (``libblosc.so.1``), so any
codec bcolz wrote (blosclz/lz4/zstd/zlib/snappy) decodes.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import functools
import json
import os
import threading
import struct
from collections import OrderedDict
from concurrent.futures import ThreadPoolExecutor

import numpy as np

BLOSCPACK_MAGIC = b'blpk'
BLOSCPACK_HEADER = 16
BLOSC_HEADER = 16
BLOSC_MAX_OVERHEAD = 16
ROOTDIRS = '__rootdirs__'
ATTRS = '__attrs__'

_BLOSC_CANDIDATES = ('/opt/conda/lib/libblosc.so.1', '/opt/conda/lib/libblosc.so', 'libblosc.so.1',
                     'libblosc.so')
_blosc = None


def blosc():
    global _blosc
    if _blosc is None:
        err = None
        for cand in _BLOSC_CANDIDATES + tuple(filter(None, [ctypes.util.find_library('blosc')])):
            try:
                lib = ctypes.CDLL(cand)
                break
            except OSError as e:
                err = e
        else:
            raise OSError('libblosc (c-blosc 1.x) not found: %s' % err)
        lib.blosc_init()
        lib.blosc_compress.restype = ctypes.c_int
        lib.blosc_compress.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.blosc_decompress.restype = ctypes.c_int
        lib.blosc_decompress.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.blosc_decompress_ctx.restype = ctypes.c_int
        lib.blosc_decompress_ctx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_int]
        lib.blosc_compress_ctx.restype = ctypes.c_int
        lib.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
        lib.blosc_cbuffer_sizes.restype = None
        lib.blosc_cbuffer_sizes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                            ctypes.POINTER(ctypes.c_size_t),
                                            ctypes.POINTER(ctypes.c_size_t)]
        _blosc = lib
    return _blosc


def _dump_json(path, obj):
    with open(path, 'wb') as f:
        f.write(json.dumps(obj, ensure_ascii=True).encode('ascii'))
        f.write(b'\n')


def _chunklen_for(itemsize, expectedlen):
    """Rows per chunk: ~1 MiB chunks for shards, at least 1 row."""
    target = 1 << 20
    return max(1, min(target // max(itemsize, 1), max(int(expectedlen), 1)))


# ------------------------------------------------------------------------------------------
# blosc frames
# ------------------------------------------------------------------------------------------
_TLS = threading.local()
_ARENA_KEEP_BYTES = 256 << 20  # result arenas up to this size stay allocated between results


def compress_chunk(arr, clevel=5, shuffle=1, cname='lz4', nthreads=1):
    arr = np.ascontiguousarray(arr)
    nbytes = arr.nbytes
    # a per-thread destination reused across calls and one copy of the compressed bytes out: a
    # fresh chunk-sized buffer per call (mmap, page faults, munmap) serialised the compression
    # pool's threads on the process's memory map
    dest = getattr(_TLS, 'dest', None)
    if dest is None or len(dest) < nbytes + BLOSC_MAX_OVERHEAD:
        dest = _TLS.dest = np.empty(max(nbytes + BLOSC_MAX_OVERHEAD, 1 << 20), np.uint8)
    n = compress_into(arr, dest, clevel, shuffle, cname, nthreads)
    return dest[:n].tobytes()


def compress_into(arr, dest, clevel=5, shuffle=1, cname='lz4', nthreads=1):
    """Compress the contiguous array ``arr`` into the uint8 array ``dest`` (at least
    arr.nbytes + BLOSC_MAX_OVERHEAD long); returns the frame's length."""
    nbytes = arr.nbytes
    n = blosc().blosc_compress_ctx(clevel, shuffle, arr.dtype.itemsize, nbytes, arr.ctypes.data, dest.ctypes.data,
                                   nbytes + BLOSC_MAX_OVERHEAD, cname.encode('ascii'), 0, nthreads)
    if n <= 0:
        raise RuntimeError('blosc compression failed (%d)' % n)
    return n


def decompress_into(frame, out_view):
    """Decode one blosc frame into the writable numpy array ``out_view``; returns bytes."""
    buf = ctypes.c_char_p(frame)
    nb, cb, bs = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    blosc().blosc_cbuffer_sizes(buf, ctypes.byref(nb), ctypes.byref(cb), ctypes.byref(bs))
    if nb.value > out_view.nbytes:
        raise ValueError('blosc frame larger than destination (%d > %d)' % (nb.value, out_view.nbytes))
    n = blosc().blosc_decompress_ctx(buf, out_view.ctypes.data, out_view.nbytes, 1)
    if n < 0:
        raise RuntimeError('blosc decompression failed (%d)' % n)
    return n


def read_blp(path):
    with open(path, 'rb') as f:
        data = f.read()
    if data[:4] != BLOSCPACK_MAGIC:
        raise ValueError('%s: not a bloscpack chunk' % path)
    return data[BLOSCPACK_HEADER:]


def bloscpack_header(nchunks=1, version=1):
    return BLOSCPACK_MAGIC + struct.pack('<B', version) + b'\x00\x00\x00' + struct.pack('<q', nchunks)


# ------------------------------------------------------------------------------------------
# carray
# ------------------------------------------------------------------------------------------
class CArrayMeta:
    def __init__(self, rootdir):
        self.rootdir = rootdir
        with open(os.path.join(rootdir, 'meta', 'sizes'), 'rb') as f:
            sizes = json.loads(f.read().decode('ascii'))
        with open(os.path.join(rootdir, 'meta', 'storage'), 'rb') as f:
            storage = json.loads(f.read().decode('ascii'))
        self.length = int(sizes['shape'][0])
        self.dtype = np.dtype(storage['dtype'])
        self.chunklen = int(storage['chunklen'])
        self.cparams = storage.get('cparams', {})
        nchunks = -(-self.length // self.chunklen) if self.length else 0
        self.chunk_files = [os.path.join(rootdir, 'data', '__%d.blp' % i) for i in range(nchunks)]


def read_carray(rootdir, out=None, pool=None):
    """Decode a carray into ``out`` (or a new array); chunks decode in parallel on ``pool``."""
    meta = CArrayMeta(rootdir)
    if out is None:
        out = np.empty(meta.length, dtype=meta.dtype)
    if meta.length == 0:
        return out

    def one(i):
        lo = i * meta.chunklen
        hi = min(meta.length, lo + meta.chunklen)
        frame = read_blp(meta.chunk_files[i])
        tmp = out[lo:hi]
        n = decompress_into(frame, tmp)
        if n != tmp.nbytes:
            raise ValueError('%s: chunk %d decoded %d bytes, expected %d' % (rootdir, i, n, tmp.nbytes))

    if pool is None or len(meta.chunk_files) < 2:
        for i in range(len(meta.chunk_files)):
            one(i)
    else:
        list(pool.map(one, range(len(meta.chunk_files))))
    return out


def _json_bytes(obj):
    return json.dumps(obj, ensure_ascii=True).encode('ascii') + b'\n'


# Compression pool: a result's chunks are compressed in parallel (libblosc releases the GIL
# through ctypes), one blosc context per chunk -- the frames are byte-identical to a serial
# compression.  bqueryd compresses results on the worker's one thread (bcolz.set_nthreads(1),
# worker.py:40): a 1 M-group result took ~29 ms of host time that way, >90 % of a C3 message.
_POOL = None
_PARALLEL_MIN_BYTES = 4 << 20


def _pool():
    global _POOL
    if _POOL is None:
        _POOL = ThreadPoolExecutor(max_workers=max(1, min(16, os.cpu_count() or 1)),
                                   thread_name_prefix='bqgpu-blosc')
    return _POOL


def carray_files(arr, chunklen=None, clevel=5, shuffle=1, cname='lz4', frames=None, parts=False):
    """The files of a carray directory: [(path relative to the carray rootdir, bytes)].
    ``frames``: the column's compressed chunks (bytes-like) when the caller already has them."""
    arr = np.ascontiguousarray(arr)
    if arr.dtype.kind not in _WRITABLE_KINDS:
        raise NotImplementedError('bcolz writer: dtype %s' % arr.dtype)
    n = len(arr)
    chunklen = chunklen or _chunklen_for(arr.dtype.itemsize, n)
    if frames is None:
        los = range(0, n, chunklen)
        comp = lambda lo: compress_chunk(arr[lo:lo + chunklen], clevel, shuffle, cname)  # noqa: E731
        frames = list(_pool().map(comp, los)) if arr.nbytes >= _PARALLEL_MIN_BYTES and len(los) > 1 else \
            [comp(lo) for lo in los]
    files = []
    cbytes = 0
    for i, frame in enumerate(frames):
        # parts=True: the file as (header, frame) -- the caller writes both without joining them
        files.append(('data/__%d.blp' % i, (bloscpack_header(1), frame) if parts else bloscpack_header(1) + frame))
        cbytes += len(frame) + BLOSCPACK_HEADER
    files.append(('meta/storage', _storage_json(arr.dtype, clevel, shuffle, cname, int(chunklen), int(max(n, 1)))))
    files.append(('meta/sizes', _json_bytes({'shape': [int(n)], 'nbytes': int(arr.nbytes), 'cbytes': int(cbytes)})))
    files.append((ATTRS, _EMPTY_ATTRS))
    return files


_EMPTY_ATTRS = b'{}\n'
# numeric, bool, fixed-width bytes / unicode and datetime64 / timedelta64 columns (the dtypes a
# bqueryd shard built with ctable.fromdataframe holds; blosc's typesize is the element size)
_WRITABLE_KINDS = 'biufSUMm'


@functools.lru_cache(maxsize=1024)
def _storage_json(dtype, clevel, shuffle, cname, chunklen, expectedlen):
    dflt = False if dtype.kind == 'b' else (0.0 if dtype.kind == 'f' else ('' if dtype.kind in 'SU' else 0))
    return _json_bytes({'dtype': str(dtype), 'cparams': {'clevel': clevel, 'shuffle': shuffle, 'cname': cname, 'quantize': 0},
                        'chunklen': chunklen, 'expectedlen': expectedlen, 'dflt': dflt})


def _write_files(rootdir, files):
    for rel, data in files:
        path = os.path.join(rootdir, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, 'wb') as f:
            f.write(data)


def write_carray(rootdir, arr, chunklen=None, clevel=5, shuffle=1, cname='lz4'):
    os.makedirs(os.path.join(rootdir, 'meta'), exist_ok=True)
    os.makedirs(os.path.join(rootdir, 'data'), exist_ok=True)
    _write_files(rootdir, carray_files(arr, chunklen, clevel, shuffle, cname))


# ------------------------------------------------------------------------------------------
# ctable
# ------------------------------------------------------------------------------------------
def ctable_names(rootdir):
    with open(os.path.join(rootdir, ROOTDIRS), 'rb') as f:
        data = json.loads(f.read().decode('ascii'))
    return [str(n) for n in data['names']]


def ctable_column_dir(rootdir, name):
    return os.path.join(rootdir, name)


def read_ctable(rootdir, columns=None, nthreads=None):
    """-> OrderedDict name -> numpy array (all columns, or the listed ones)."""
    names = ctable_names(rootdir)
    if columns is None:
        columns = names
    for c in columns:
        if c not in names:
            raise KeyError(str(c))
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    # small tables (query results: a few chunks) decode inline -- a thread pool costs more
    nchunks = sum(len(CArrayMeta(ctable_column_dir(rootdir, c)).chunk_files) for c in columns)
    out = OrderedDict()
    if nthreads <= 1 or nchunks <= 2 * len(columns):
        for c in columns:
            out[c] = read_carray(ctable_column_dir(rootdir, c))
        return out
    with ThreadPoolExecutor(max_workers=min(nthreads, nchunks)) as pool:
        for c in columns:
            out[c] = read_carray(ctable_column_dir(rootdir, c), pool=pool)
    return out


def ctable_len(rootdir):
    names = ctable_names(rootdir)
    if not names:
        return 0
    return CArrayMeta(ctable_column_dir(rootdir, names[0])).length


def ctable_dtypes(rootdir):
    return OrderedDict((n, CArrayMeta(ctable_column_dir(rootdir, n)).dtype) for n in ctable_names(rootdir))


def ctable_files(columns, chunklen=None, cname='lz4'):
    """The files of a ctable rootdir: [(relative path, bytes)], column directories first."""
    names = list(columns.keys())
    files = []
    for n in names:
        files += [(n + '/' + rel, data) for rel, data in carray_files(columns[n], chunklen=chunklen, cname=cname)]
    files.append((ROOTDIRS, _json_bytes({'names': names, 'dirs': {n: n for n in names}})))
    files.append((ATTRS, _json_bytes({})))
    return files


def write_ctable(rootdir, columns, chunklen=None, cname='lz4'):
    """Write an OrderedDict of equal-length arrays as a bcolz ctable rootdir."""
    os.makedirs(rootdir, exist_ok=True)
    for n in columns:  # bcolz creates both even for a zero-row column (no chunk file)
        os.makedirs(os.path.join(rootdir, n, 'data'), exist_ok=True)
        os.makedirs(os.path.join(rootdir, n, 'meta'), exist_ok=True)
    _write_files(rootdir, ctable_files(columns, chunklen, cname))
    return rootdir


_TAR_IDS = b'0000000\x00' * 2          # uid, gid
_TAR_MAGIC = b'ustar\x0000'             # magic + version
_TAR_DEVS = bytes(16)                    # devmajor, devminor: empty unless a device file
_TAR_FIXED_SUM = sum(_TAR_IDS) + sum(b' ' * 8) + sum(_TAR_MAGIC) + sum(_TAR_DEVS)


_TAR_TAIL = bytes(100) + _TAR_MAGIC + bytes(64) + _TAR_DEVS + bytes(167)  # after the type flag


def _tar_header(name, size, mode, mtime, dirtype):
    """One 512-byte ustar header exactly as ``tarfile`` (default PAX format, a name of at most
    100 bytes: no extended header) writes it for a TarInfo with uid / gid 0 and empty owner
    names."""
    nb = name.encode('utf-8')
    if len(nb) > 100:
        raise ValueError('tar member name longer than 100 bytes: %s' % name)
    m, sz, mt = b'%07o\x00' % mode, b'%011o\x00' % size, b'%011o\x00' % mtime
    typ = b'5' if dirtype else b'0'  # directory / regular file
    # checksum: every byte of the header with the checksum field read as spaces
    cks = _TAR_FIXED_SUM + sum(nb) + sum(m) + sum(sz) + sum(mt) + typ[0]
    return nb.ljust(100, b'\x00') + m + _TAR_IDS + sz + mt + (b'%06o\x00 ' % cks) + typ + _TAR_TAIL


def ctable_tar(columns, arcname, chunklen=None, cname='lz4'):
    """Bytes of ``tarfile.open(mode='w').add(<ctable rootdir>, arcname=arcname)``
    (worker.py:337-345), built in memory: the same members as ``write_ctable`` + ``tarfile.add``
    (the directory, then its entries sorted by name, depth first; every column has data/ and
    meta/ even when a zero-row column has no chunk file -- the client appends to the first
    result it opens, rpc.py:158-162, and bcolz then writes chunks into data/) without writing
    the ctable to disk.  The ustar blocks are written directly (``_tar_header``, byte-identical
    to ``tarfile``'s, which took most of a warm per-file message's host time)."""
    import time
    now = int(time.time())
    out = []

    def member(name, data):
        parts = data if isinstance(data, tuple) else (data,)
        size = sum(len(d) for d in parts)
        out.append(_tar_header(name, size, 0o644, now, False))
        out.extend(parts)
        if size % 512:
            out.append(bytes(512 - size % 512))

    def directory(name):
        out.append(_tar_header(name + '/', 0, 0o755, now, True))

    names = list(columns.keys())
    # every column's chunks, compressed on the pool when the result is large
    arrays = {n: np.ascontiguousarray(columns[n]) for n in names}
    for n, a in arrays.items():
        if a.dtype.kind not in _WRITABLE_KINDS:
            raise NotImplementedError('bcolz writer: dtype %s' % a.dtype)
    clen = {n: chunklen or _chunklen_for(a.dtype.itemsize, len(a)) for n, a in arrays.items()}
    jobs = [(n, lo) for n in names for lo in range(0, len(arrays[n]), clen[n])]
    total = sum(a.nbytes for a in arrays.values())

    # every frame compressed straight into one arena, kept per calling thread and reused (per-
    # frame buffers cost each pool thread an mmap / munmap pair and page faults on a fresh
    # buffer, which serialise on the process's memory map) and handed to the tar as views of it
    # -- the join below copies them out before the arena is used again
    offs, o = [], 0
    for n, lo in jobs:
        offs.append(o)
        o += min(clen[n], len(arrays[n]) - lo) * arrays[n].dtype.itemsize + BLOSC_MAX_OVERHEAD
    arena = getattr(_TLS, 'arena', None)
    if arena is None or len(arena) < o:
        arena = np.empty(max(o, 1 << 20), np.uint8)
        if o <= _ARENA_KEEP_BYTES:
            _TLS.arena = arena
    view = memoryview(arena)

    def comp(i):
        n, lo = jobs[i]
        a = arrays[n][lo:lo + clen[n]]
        return compress_into(a, arena[offs[i]:offs[i] + a.nbytes + BLOSC_MAX_OVERHEAD], 5, 1, cname)

    idx = range(len(jobs))
    done = list(_pool().map(comp, idx)) if total >= _PARALLEL_MIN_BYTES and len(jobs) > 1 else [comp(i) for i in idx]
    frames = {n: [] for n in names}
    for i, ((n, _), f) in enumerate(zip(jobs, done)):
        frames[n].append(view[offs[i]:offs[i] + f])
    root = {ATTRS: _json_bytes({}), ROOTDIRS: _json_bytes({'names': names, 'dirs': {n: n for n in names}})}
    directory(arcname)
    for entry in sorted(list(root) + names):
        if entry in root and entry not in columns:
            member(arcname + '/' + entry, root[entry])
            continue
        files = dict(carray_files(arrays[entry], chunklen=clen[entry], cname=cname, frames=frames[entry], parts=True))
        cdir = arcname + '/' + entry
        directory(cdir)
        member(cdir + '/' + ATTRS, files.pop(ATTRS))
        directory(cdir + '/data')  # '__attrs__' < 'data' < 'meta'
        for rel in sorted(r for r in files if r.startswith('data/')):
            member(cdir + '/' + rel, files[rel])
        directory(cdir + '/meta')
        member(cdir + '/meta/sizes', files['meta/sizes'])
        member(cdir + '/meta/storage', files['meta/storage'])
    out.append(bytes(1024))  # end-of-archive: two zero blocks
    body = b''.join(out)
    return body + bytes(-len(body) % 10240)  # tarfile pads the archive to whole 20-block records


def read_ctable_files(files, columns=None):
    """A ctable from its files in memory ({relative path: bytes}, e.g. a result tar's
    members with the top directory stripped) -> OrderedDict name -> numpy array."""
    names = [str(n) for n in json.loads(files[ROOTDIRS].decode('ascii'))['names']]
    out = OrderedDict()
    for n in (columns or names):
        if n not in names:
            raise KeyError(str(n))
        sizes = json.loads(files[n + '/meta/sizes'].decode('ascii'))
        storage = json.loads(files[n + '/meta/storage'].decode('ascii'))
        length, chunklen = int(sizes['shape'][0]), int(storage['chunklen'])
        arr = np.empty(length, dtype=np.dtype(storage['dtype']))
        for i, lo in enumerate(range(0, length, chunklen)):
            data = files[n + '/data/__%d.blp' % i]
            if data[:4] != BLOSCPACK_MAGIC:
                raise ValueError('%s chunk %d: not a bloscpack chunk' % (n, i))
            tmp = arr[lo:lo + chunklen]
            if decompress_into(data[BLOSCPACK_HEADER:], tmp) != tmp.nbytes:
                raise ValueError('%s chunk %d: short chunk' % (n, i))
        out[n] = arr
    return out
