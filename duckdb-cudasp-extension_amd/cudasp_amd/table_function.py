"""cudasp_scan(...) -- the reference's SQL table function, driven from Python.

This is a thin ctypes driver of the C++ table-function host
(csrc/host/cudasp_host.cpp, ABI include/cudasp_host.h) playing the role of
DuckDB's executor: it binds the arguments (same validation and messages as
CudaspScanBind, src/cudasp_extension.cu:420-509), feeds the input table to one
local state per "executor thread" in DuckDB-sized chunks of <= 2048 rows
(CudaspScanFunction :534-552), then finalizes every thread; the last one emits
the matches (CudaspScanFinalFunction :554-624).

    rows = [(txid: bytes, height: int, tweak_key: bytes(64), outputs: [int|None] | None), ...]
    cudasp_scan(rows, scan_private_key, spend_public_key, label_keys, batch_size=...)
      -> [(txid, height, tweak_key), ...]   (order unspecified, like the reference)
"""
import ctypes
import threading

from . import _native

VECTOR_SIZE = 2048
TF_HAVE_MORE_OUTPUT = 1


class InvalidInputException(ValueError):
    """Raised with the reference's InvalidInputException messages."""


class _BlobArg(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("size", ctypes.c_uint64), ("is_blob", ctypes.c_int)]


class _Chunk(ctypes.Structure):
    _fields_ = [
        ("count", ctypes.c_uint32),
        ("txid_data", ctypes.POINTER(ctypes.c_void_p)),
        ("txid_size", ctypes.POINTER(ctypes.c_uint32)),
        ("txid_valid", ctypes.POINTER(ctypes.c_uint8)),
        ("height", ctypes.POINTER(ctypes.c_int32)),
        ("height_valid", ctypes.POINTER(ctypes.c_uint8)),
        ("tweak_data", ctypes.POINTER(ctypes.c_void_p)),
        ("tweak_size", ctypes.POINTER(ctypes.c_uint32)),
        ("tweak_valid", ctypes.POINTER(ctypes.c_uint8)),
        ("list_offset", ctypes.POINTER(ctypes.c_uint64)),
        ("list_length", ctypes.POINTER(ctypes.c_uint64)),
        ("list_valid", ctypes.POINTER(ctypes.c_uint8)),
        ("child_values", ctypes.POINTER(ctypes.c_int64)),
        ("child_valid", ctypes.POINTER(ctypes.c_uint8)),
        ("child_blob_data", ctypes.POINTER(ctypes.c_void_p)),
        ("child_blob_size", ctypes.POINTER(ctypes.c_uint32)),
    ]


class _Vector(ctypes.Structure):
    """cudasp_tf_vector (include/cudasp_host.h): a DuckDB UnifiedVectorFormat."""
    _fields_ = [("data", ctypes.c_void_p), ("sel", ctypes.c_void_p), ("validity", ctypes.c_void_p)]


class _Vectors(ctypes.Structure):
    """cudasp_tf_vectors (include/cudasp_host.h)."""
    _fields_ = [("count", ctypes.c_uint32), ("txid", _Vector), ("height", _Vector), ("tweak", _Vector),
                ("outputs", _Vector), ("child", _Vector)]


STRING_INLINE = 12  # string_t::INLINE_LENGTH


class _Output(ctypes.Structure):
    _fields_ = [
        ("count", ctypes.c_uint32),
        ("txid_data", ctypes.c_void_p * VECTOR_SIZE),
        ("txid_size", ctypes.c_uint32 * VECTOR_SIZE),
        ("height", ctypes.c_int32 * VECTOR_SIZE),
        ("tweak_data", ctypes.c_void_p * VECTOR_SIZE),
        ("tweak_size", ctypes.c_uint32 * VECTOR_SIZE),
    ]


class _Columns(ctypes.Structure):
    _fields_ = [
        ("count", ctypes.c_uint64),
        ("txid_offsets", ctypes.c_void_p),
        ("txid_data", ctypes.c_void_p),
        ("txid_validity", ctypes.c_void_p),
        ("txid_offset", ctypes.c_uint64),
        ("height", ctypes.c_void_p),
        ("height_validity", ctypes.c_void_p),
        ("height_offset", ctypes.c_uint64),
        ("tweak_offsets", ctypes.c_void_p),
        ("tweak_data", ctypes.c_void_p),
        ("tweak_validity", ctypes.c_void_p),
        ("tweak_offset", ctypes.c_uint64),
        ("tweak_fixed_width", ctypes.c_int32),
        ("list_offsets", ctypes.c_void_p),
        ("list_validity", ctypes.c_void_p),
        ("list_offset", ctypes.c_uint64),
        ("child_values", ctypes.c_void_p),
        ("child_validity", ctypes.c_void_p),
        ("child_offset", ctypes.c_uint64),
        ("child_blob_offsets", ctypes.c_void_p),
        ("child_blob_data", ctypes.c_void_p),
        ("child_blob_fixed_width", ctypes.c_int32),
    ]


class _Stats(ctypes.Structure):
    _fields_ = [
        ("feeds", ctypes.c_uint32),
        ("streams_per_feed", ctypes.c_uint32),
        ("max_streams_per_device", ctypes.c_uint32),
        ("hw_queues", ctypes.c_uint32),
        ("launches", ctypes.c_uint64),
        ("rows", ctypes.c_uint64),
        ("harvest_wait_s", ctypes.c_double),
        ("reserve_s", ctypes.c_double),
        ("copy_s", ctypes.c_double),
        ("launch_s", ctypes.c_double),
        ("streaming_feeds", ctypes.c_uint32),
    ]


class _PinnedInfo(ctypes.Structure):
    """cudasp_pinned_info_t (include/cudasp_host.h)."""
    _fields_ = [
        ("rows_appended", ctypes.c_uint64),
        ("rows_pinned", ctypes.c_uint64),
        ("batches", ctypes.c_uint64),
        ("pinned_bytes", ctypes.c_uint64),
        ("last_matches", ctypes.c_uint64),
        ("last_scan_s", ctypes.c_double),
        ("last_publish_s", ctypes.c_double),
        ("placement", ctypes.c_int32),
        ("device_bytes", ctypes.c_uint64),
    ]


def _read_stats(lib, g, stats):
    """Fill the dict `stats` from cudasp_tf_get_stats (after the last final)."""
    if stats is None:
        return
    st = _Stats()
    _native.check(lib.cudasp_tf_get_stats(g, ctypes.byref(st)))
    stats.update({name: getattr(st, name) for name, _ in _Stats._fields_})


_P = ctypes.c_void_p
_HOST_SIGNATURES = {
    "cudasp_tf_bind": (ctypes.c_int, [ctypes.c_uint32, _BlobArg, _BlobArg, ctypes.c_int, ctypes.POINTER(_BlobArg),
                                      ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                      ctypes.POINTER(_P), ctypes.c_char_p, ctypes.c_size_t]),
    "cudasp_tf_bind_options": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]),
    "cudasp_tf_bind_free": (None, [_P]),
    "cudasp_tf_bind_batch_size": (ctypes.c_uint64, [_P]),
    "cudasp_tf_init": (ctypes.c_int, [_P, ctypes.POINTER(_P)]),
    "cudasp_tf_global_free": (None, [_P]),
    "cudasp_tf_num_gpus": (ctypes.c_int, [_P]),
    "cudasp_tf_local_init": (ctypes.c_int, [_P, ctypes.POINTER(_P)]),
    "cudasp_tf_local_free": (None, [_P]),
    "cudasp_tf_local_gpu": (ctypes.c_int, [_P]),
    "cudasp_tf_local_device": (ctypes.c_int, [_P]),
    "cudasp_assign_gpu": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32]),
    "cudasp_tf_release_pool": (None, []),
    "cudasp_tf_pool_size": (ctypes.c_uint32, []),
    "cudasp_tf_function": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(_Chunk)]),
    "cudasp_tf_function_vectors": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(_Vectors)]),
    "cudasp_tf_prewarm": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(ctypes.c_double)]),
    "cudasp_tf_final": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(_Output)]),
    "cudasp_tf_function_columns": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(_Columns)]),
    "cudasp_tf_get_stats": (ctypes.c_int, [_P, ctypes.POINTER(_Stats)]),
    "cudasp_pinned_create": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(ctypes.c_int), ctypes.c_uint32,
                                            ctypes.POINTER(_P)]),
    "cudasp_pinned_create_placed": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(ctypes.c_int), ctypes.c_uint32,
                                                   ctypes.c_int, ctypes.POINTER(_P)]),
    "cudasp_pinned_append": (ctypes.c_int, [_P, ctypes.POINTER(_Columns)]),
    "cudasp_pinned_scan": (ctypes.c_int, [_P, _P, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                          ctypes.POINTER(ctypes.c_uint64)]),
    "cudasp_pinned_free_rows": (None, [ctypes.POINTER(ctypes.c_uint64)]),
    "cudasp_pinned_info": (ctypes.c_int, [_P, ctypes.POINTER(_PinnedInfo)]),
    "cudasp_pinned_free": (None, [_P]),
}

_host = None


def _lib():
    global _host
    if _host is None:
        lib = _native.load()
        for name, (res, args) in _HOST_SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _host = lib
    return _host


def _blob(value):
    """(keep-alive, _BlobArg) for a Python value; bytes-like = BLOB."""
    if isinstance(value, (bytes, bytearray, memoryview)):
        buf = ctypes.create_string_buffer(bytes(value), max(1, len(value)))
        return buf, _BlobArg(ctypes.cast(buf, ctypes.c_void_p), len(value), 1)
    return None, _BlobArg(None, 0, 0)


class BoundScan:
    """Bind data of one cudasp_scan call (CudaspScanBindData)."""

    def __init__(self, scan_private_key, spend_public_key, label_keys, batch_size=None, arg_count=4,
                 output_count=None, label_negation=None, full_x=None):
        lib = _lib()
        keep = []
        k1, a1 = _blob(scan_private_key)
        k2, a2 = _blob(spend_public_key)
        keep += [k1, k2]
        is_list = isinstance(label_keys, (list, tuple))
        labels = list(label_keys) if is_list else []
        arr = (_BlobArg * max(1, len(labels)))()
        for i, l in enumerate(labels):
            k, arr[i] = _blob(l)
            keep.append(k)
        has_bs = batch_size is not None
        bs_int = isinstance(batch_size, int) and not isinstance(batch_size, bool)
        err = ctypes.create_string_buffer(512)
        h = _P()
        rc = lib.cudasp_tf_bind(arg_count, a1, a2, 1 if is_list else 0, arr, len(labels), 1 if has_bs else 0,
                                1 if bs_int else 0, int(batch_size) if bs_int else 0, ctypes.byref(h), err, 512)
        if rc != 0:
            raise InvalidInputException(err.value.decode())
        self._h = h
        self.batch_size = lib.cudasp_tf_bind_batch_size(h)
        # named parameters of the protocol variants (None = not given)
        rc = lib.cudasp_tf_bind_options(h, output_count is not None, int(output_count or 0),
                                        label_negation is not None, bool(label_negation), full_x is not None,
                                        bool(full_x), err, 512)
        if rc != 0:
            raise InvalidInputException(err.value.decode())
        self.full_x = bool(full_x)

    def __del__(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib().cudasp_tf_bind_free(self._h)
            self._h = None


def _make_chunk(rows, full_x=False):
    """Build a DuckDB-like unified chunk from Python rows; returns (keep, chunk).
    With full_x the outputs are BLOB lists (32-byte x-only keys)."""
    n = len(rows)
    keep = []
    txid_ptrs = (ctypes.c_void_p * n)()
    txid_size = (ctypes.c_uint32 * n)()
    txid_valid = (ctypes.c_uint8 * n)()
    height = (ctypes.c_int32 * n)()
    height_valid = (ctypes.c_uint8 * n)()
    tweak_ptrs = (ctypes.c_void_p * n)()
    tweak_size = (ctypes.c_uint32 * n)()
    tweak_valid = (ctypes.c_uint8 * n)()
    list_offset = (ctypes.c_uint64 * n)()
    list_length = (ctypes.c_uint64 * n)()
    list_valid = (ctypes.c_uint8 * n)()
    child = []
    child_ok = []
    for i, (txid, h, tweak, outs) in enumerate(rows):
        if txid is not None:
            b = ctypes.create_string_buffer(bytes(txid), max(1, len(txid)))
            keep.append(b)
            txid_ptrs[i] = ctypes.cast(b, ctypes.c_void_p)
            txid_size[i] = len(txid)
            txid_valid[i] = 1
        if h is not None:
            height[i] = h
            height_valid[i] = 1
        if tweak is not None:
            b = ctypes.create_string_buffer(bytes(tweak), max(1, len(tweak)))
            keep.append(b)
            tweak_ptrs[i] = ctypes.cast(b, ctypes.c_void_p)
            tweak_size[i] = len(tweak)
            tweak_valid[i] = 1
        list_offset[i] = len(child)
        if outs is not None:
            list_valid[i] = 1
            list_length[i] = len(outs)
            for o in outs:
                child.append(o if full_x else (0 if o is None else o))
                child_ok.append(0 if o is None else 1)
    cvalid = (ctypes.c_uint8 * max(1, len(child_ok)))(*child_ok)
    if full_x:
        cv = None
        bdata = (ctypes.c_void_p * max(1, len(child)))()
        bsize = (ctypes.c_uint32 * max(1, len(child)))()
        for i, o in enumerate(child):
            if o is not None:
                b = ctypes.create_string_buffer(bytes(o), max(1, len(o)))
                keep.append(b)
                bdata[i] = ctypes.cast(b, ctypes.c_void_p)
                bsize[i] = len(o)
        keep += [bdata, bsize]
    else:
        cv = (ctypes.c_int64 * max(1, len(child)))(*child)
        bdata, bsize = None, None
    keep += [txid_ptrs, txid_size, txid_valid, height, height_valid, tweak_ptrs, tweak_size, tweak_valid,
             list_offset, list_length, list_valid, cv, cvalid]
    c = _Chunk(n, txid_ptrs, txid_size, txid_valid, height, height_valid, tweak_ptrs, tweak_size, tweak_valid,
               list_offset, list_length, list_valid, cv, cvalid, bdata, bsize)
    return keep, c


def _make_vectors(rows, full_x=False, rng=None):
    """DuckDB's vectors for Python rows (cudasp_tf_vectors), as a DataChunk
    holds them: 16-byte string_t (bytes inline up to 12, else prefix +
    pointer), int32 heights, list_entry_t lists into one child vector, 64-bit
    validity words.  With `rng` (a numpy Generator) every vector -- the child
    too -- is stored in a shuffled physical order behind a selection vector,
    as a dictionary or filtered vector reaches an operator.  Returns (keep,
    vectors)."""
    import numpy as np
    n = len(rows)
    keep = []

    def perm(m):
        return rng.permutation(m).astype(np.uint32) if rng is not None else None

    def vec(values, ok, kind):
        """(data, sel, validity) arrays for one column in a physical order."""
        m = len(values)
        sel = perm(m)
        pos = sel if sel is not None else np.arange(m, dtype=np.uint32)  # logical i -> physical pos[i]
        words = np.zeros(max(1, (m + 63) // 64), dtype=np.uint64)
        if kind == "str":
            data = np.zeros((max(1, m), 16), dtype=np.uint8)
        elif kind == "i32":
            data = np.zeros(max(1, m), dtype=np.int32)
        elif kind == "i64":
            data = np.zeros(max(1, m), dtype=np.int64)
        else:  # list entries
            data = np.zeros((max(1, m), 2), dtype=np.uint64)
        for i, (v, good) in enumerate(zip(values, ok)):
            p = int(pos[i])
            if not good:
                continue
            words[p >> 6] |= np.uint64(1) << np.uint64(p & 63)
            if kind == "str":
                b = bytes(v)
                data[p, 0:4] = np.frombuffer(np.uint32(len(b)).tobytes(), np.uint8)
                if len(b) <= STRING_INLINE:
                    data[p, 4:4 + len(b)] = np.frombuffer(b, np.uint8) if b else 0
                else:
                    buf = ctypes.create_string_buffer(b, len(b))
                    keep.append(buf)
                    data[p, 4:8] = np.frombuffer(b[:4], np.uint8)
                    data[p, 8:16] = np.frombuffer(np.uint64(ctypes.addressof(buf)).tobytes(), np.uint8)
            elif kind == "list":
                data[p] = v
            else:
                data[p] = v
        keep.extend([data, words] + ([sel] if sel is not None else []))
        return _Vector(data.ctypes.data, sel.ctypes.data if sel is not None else None,
                       words.ctypes.data if not all(ok) else None)

    child, child_ok, entries = [], [], []
    for txid, h, tweak, outs in rows:
        entries.append((len(child), len(outs) if outs is not None else 0))
        for o in outs or []:
            child.append(o if o is not None else (b"" if full_x else 0))
            child_ok.append(o is not None)
    v = _Vectors()
    v.count = n
    v.txid = vec([r[0] or b"" for r in rows], [r[0] is not None for r in rows], "str")
    v.height = vec([r[1] or 0 for r in rows], [r[1] is not None for r in rows], "i32")
    v.tweak = vec([r[2] or b"" for r in rows], [r[2] is not None for r in rows], "str")
    v.outputs = vec(entries, [r[3] is not None for r in rows], "list")
    v.child = vec(child, child_ok, "str" if full_x else "i64")
    return keep, v


def assign_gpu(ordinal, num_gpus):
    """The product's multi-GPU work assignment (cudasp_assign_gpu,
    include/cudasp_host.h): unit `ordinal` -> GPU ordinal mod num_gpus, as
    the host assigns executor threads (src/cudasp_extension.cu:523-529) and
    bench.py assigns the batches of one table to ranks.  Host-only."""
    return int(_lib().cudasp_assign_gpu(int(ordinal), int(num_gpus)))


def pool_size():
    """GPU contexts parked in the host's cross-query pool (cudasp_tf_pool_size)."""
    return int(_lib().cudasp_tf_pool_size())


def prewarm(batch_size=0):
    """Build the fixed-base tables and park one ready streaming feed per GPU
    (cudasp_tf_prewarm); returns the seconds it took."""
    secs = ctypes.c_double()
    _native.check(_lib().cudasp_tf_prewarm(int(batch_size), ctypes.byref(secs)))
    return secs.value


def release_pool():
    """Free the host's pooled GPU contexts (cudasp_tf_release_pool)."""
    _lib().cudasp_tf_release_pool()


def cudasp_scan(rows, scan_private_key, spend_public_key, label_keys, batch_size=None, threads=1,
                chunk_rows=VECTOR_SIZE, output_count=None, label_negation=None, full_x=None, assignments=None,
                stats=None, input="rows", seed=None):
    """Run the table function over `rows` with `threads` executor threads.
    Chunks are dealt round-robin to the threads, as DuckDB's parallel scan
    would hand out morsels; each thread gets its own local state (and GPU,
    round-robin, CudaspScanLocalInit :523-529).  output_count /
    label_negation / full_x: the protocol-variant named parameters
    (cudasp_tf_bind_options); with full_x the outputs are lists of 32-byte
    x-only keys.  assignments: if a list, receives (logical GPU, HIP device)
    of each thread's local state.  stats: if a dict, receives the query's
    host statistics (cudasp_tf_get_stats: feeds, streams, launches, rows,
    harvest wait).  input: "rows" hands each chunk over as per-row pointers
    (cudasp_tf_function), "vectors" as DuckDB's own vectors
    (cudasp_tf_function_vectors: string_t, list_entry_t, validity words; with
    `seed`, every vector behind a shuffled selection vector)."""
    lib = _lib()
    bound = BoundScan(scan_private_key, spend_public_key, label_keys, batch_size, output_count=output_count,
                      label_negation=label_negation, full_x=full_x)
    g = _P()
    _native.check(lib.cudasp_tf_init(bound._h, ctypes.byref(g)))
    locals_ = []
    try:
        for _ in range(threads):
            l = _P()
            _native.check(lib.cudasp_tf_local_init(g, ctypes.byref(l)))
            locals_.append(l)
            if assignments is not None:
                assignments.append((int(lib.cudasp_tf_local_gpu(l)), int(lib.cudasp_tf_local_device(l))))
        chunks = [rows[i:i + chunk_rows] for i in range(0, len(rows), chunk_rows)]
        errors = []
        results = []
        res_lock = threading.Lock()

        def worker(t):
            try:
                for ci in range(t, len(chunks), threads):
                    if input == "vectors":
                        import numpy as np
                        rng = np.random.default_rng([seed, ci]) if seed is not None else None
                        keep, c = _make_vectors(chunks[ci], bound.full_x, rng)
                        rc = lib.cudasp_tf_function_vectors(bound._h, g, locals_[t], ctypes.byref(c))
                    else:
                        keep, c = _make_chunk(chunks[ci], bound.full_x)
                        rc = lib.cudasp_tf_function(bound._h, g, locals_[t], ctypes.byref(c))
                    if rc < 0:
                        _native.check(rc)
                out = _Output()
                while True:
                    rc = lib.cudasp_tf_final(bound._h, g, locals_[t], ctypes.byref(out))
                    if rc < 0:
                        _native.check(rc)
                    got = []
                    for i in range(out.count):
                        got.append((ctypes.string_at(out.txid_data[i], out.txid_size[i]), out.height[i],
                                    ctypes.string_at(out.tweak_data[i], out.tweak_size[i])))
                    with res_lock:
                        results.extend(got)
                    if rc != TF_HAVE_MORE_OUTPUT:
                        break
            except Exception as e:  # surfaced after join
                errors.append(e)

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        if errors:
            raise errors[0]
        _read_stats(lib, g, stats)
        return results
    finally:
        for l in locals_:
            lib.cudasp_tf_local_free(l)
        lib.cudasp_tf_global_free(g)


# ------------------------------------------------------------ Arrow columns
def _addr(buf):
    return None if buf is None else buf.address


def _arrow_pieces(data, piece_rows, full_x=False):
    """Record batches of `data` (pa.Table, pa.RecordBatch or an iterable of
    record batches), columns cast to the layouts cudasp_tf_columns takes,
    sliced into pieces of at most piece_rows rows."""
    import pyarrow as pa
    if isinstance(data, pa.Table):
        batches = data.to_batches()
    elif isinstance(data, pa.RecordBatch):
        batches = [data]
    else:
        batches = list(data)
    out = []
    for rb in batches:
        if rb.num_columns < 4:
            raise InvalidInputException("cudasp_scan input needs 4 columns (txid, height, tweak_key, outputs)")
        txid, height, tweak, outs = (rb.column(i) for i in range(4))
        if not pa.types.is_binary(txid.type):
            txid = txid.cast(pa.binary())
        if not pa.types.is_int32(height.type):
            height = height.cast(pa.int32())
        if not (pa.types.is_binary(tweak.type) or pa.types.is_fixed_size_binary(tweak.type)):
            tweak = tweak.cast(pa.binary())
        if full_x:
            vt = outs.type.value_type if pa.types.is_list(outs.type) else None
            if not (vt is not None and (pa.types.is_binary(vt) or pa.types.is_fixed_size_binary(vt))):
                outs = outs.cast(pa.list_(pa.binary()))
        elif not (pa.types.is_list(outs.type) and pa.types.is_int64(outs.type.value_type)):
            outs = outs.cast(pa.list_(pa.int64()))
        for start in range(0, len(txid), piece_rows):
            m = min(piece_rows, len(txid) - start)
            out.append((txid.slice(start, m), height.slice(start, m), tweak.slice(start, m), outs.slice(start, m)))
    return out


def _columns(txid, height, tweak, outs):
    """cudasp_tf_columns over pyarrow arrays (buffers stay owned by the arrays)."""
    import pyarrow as pa
    c = _Columns()
    c.count = len(txid)
    tb = txid.buffers()
    c.txid_validity, c.txid_offsets, c.txid_data = _addr(tb[0]) if txid.null_count else None, _addr(tb[1]), _addr(tb[2])
    c.txid_offset = txid.offset
    hb = height.buffers()
    c.height_validity, c.height = _addr(hb[0]) if height.null_count else None, _addr(hb[1])
    c.height_offset = height.offset
    wb = tweak.buffers()
    c.tweak_validity = _addr(wb[0]) if tweak.null_count else None
    if pa.types.is_fixed_size_binary(tweak.type):
        c.tweak_offsets, c.tweak_data, c.tweak_fixed_width = None, _addr(wb[1]), tweak.type.byte_width
    else:
        c.tweak_offsets, c.tweak_data, c.tweak_fixed_width = _addr(wb[1]), _addr(wb[2]), 0
    c.tweak_offset = tweak.offset
    lb = outs.buffers()
    c.list_validity, c.list_offsets = _addr(lb[0]) if outs.null_count else None, _addr(lb[1])
    c.list_offset = outs.offset
    child = outs.values
    cb = child.buffers()
    c.child_validity = _addr(cb[0]) if child.null_count else None
    c.child_offset = child.offset
    if pa.types.is_fixed_size_binary(child.type):
        c.child_blob_data, c.child_blob_fixed_width = _addr(cb[1]), child.type.byte_width
    elif pa.types.is_binary(child.type):
        c.child_blob_offsets, c.child_blob_data = _addr(cb[1]), _addr(cb[2])
    else:
        c.child_values = _addr(cb[1])
    return c


def cudasp_scan_arrow(data, scan_private_key, spend_public_key, label_keys, batch_size=None, threads=1,
                      piece_rows=65536, output_count=None, label_negation=None, full_x=None, stats=None):
    """cudasp_scan over Arrow data (a pyarrow Table / RecordBatch / iterable of
    record batches, e.g. pyarrow.parquet.read_table(...) or DuckDB's
    .arrow()), with the same four columns by position.  Rows reach the
    batch buffers through cudasp_tf_function_columns (bulk copies from the
    Arrow buffers); the semantics and batches equal cudasp_scan's.  Returns a
    pyarrow Table (txid binary, height int32, tweak_key binary) in unspecified
    row order, like the reference.  output_count / label_negation / full_x /
    stats as for cudasp_scan (full_x: outputs list<binary> or
    list<fixed_size_binary(32)>)."""
    import pyarrow as pa
    lib = _lib()
    bound = BoundScan(scan_private_key, spend_public_key, label_keys, batch_size, output_count=output_count,
                      label_negation=label_negation, full_x=full_x)
    pieces = _arrow_pieces(data, piece_rows, bound.full_x)
    g = _P()
    _native.check(lib.cudasp_tf_init(bound._h, ctypes.byref(g)))
    locals_ = []
    try:
        for _ in range(threads):
            l = _P()
            _native.check(lib.cudasp_tf_local_init(g, ctypes.byref(l)))
            locals_.append(l)
        errors = []
        results = []
        res_lock = threading.Lock()

        def worker(t):
            try:
                for pi in range(t, len(pieces), threads):
                    cols = _columns(*pieces[pi])
                    rc = lib.cudasp_tf_function_columns(bound._h, g, locals_[t], ctypes.byref(cols))
                    if rc < 0:
                        _native.check(rc)
                out = _Output()
                while True:
                    rc = lib.cudasp_tf_final(bound._h, g, locals_[t], ctypes.byref(out))
                    if rc < 0:
                        _native.check(rc)
                    got = [(ctypes.string_at(out.txid_data[i], out.txid_size[i]), out.height[i],
                            ctypes.string_at(out.tweak_data[i], out.tweak_size[i])) for i in range(out.count)]
                    with res_lock:
                        results.extend(got)
                    if rc != TF_HAVE_MORE_OUTPUT:
                        break
            except Exception as e:  # surfaced after join
                errors.append(e)

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        if errors:
            raise errors[0]
        _read_stats(lib, g, stats)
        return pa.table({"txid": pa.array([r[0] for r in results], pa.binary()),
                         "height": pa.array([r[1] for r in results], pa.int32()),
                         "tweak_key": pa.array([r[2] for r in results], pa.binary())})
    finally:
        for l in locals_:
            lib.cudasp_tf_local_free(l)
        lib.cudasp_tf_global_free(g)
