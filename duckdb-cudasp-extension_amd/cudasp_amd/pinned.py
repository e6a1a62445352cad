"""A tweak table held in coherent pinned host memory and scanned in place.

The reference copies every row of every query into per-thread strings and
managed buffers (src/cudasp_extension.cu:188-223, 327-337); the table-function
host (include/cudasp_host.h) still copies each chunk into its batch slots,
which is the host's cost per row.  A tweak table is
static while wallets (scan keys) come and go, so PinnedTable copies it ONCE
into pinned memory (cudasp_host_alloc), laid out as the streaming kernel reads
it -- 64-byte tweak blobs, the outputs list's int64 values and Arrow-style
offsets (n + 1 per batch: cudasp_stream_batch with output_lengths NULL) -- and
every scan() publishes those buffers to one persistent k_scan_stream as they
are: no host copy per query, the GPU reads the rows over PCIe in place.

Same inputs and semantics as cudasp_scan_arrow (columns by position: txid
BLOB, height INTEGER, tweak_key BLOB(64), outputs BIGINT[]; rows with a NULL
txid, height or tweak are skipped, a NULL list scans as empty, NULL list
elements are dropped, a tweak of another size is an error), output_count and
label_negation included (not full_x); results as a pyarrow Table (txid,
height, tweak_key), row order unspecified like the reference's.
"""
import time

import numpy as np

from ._native import CudaspError
from .scanner import HostBuffer, Scanner, ScanStream
from .table_function import BoundScan, InvalidInputException

STREAM_RING = 64  # batches in flight at most (include/cudasp_abi.h)
ERR_INVALID_ARG, ERR_CAPACITY = -2, -5  # CUDASP_ERR_* (include/cudasp_abi.h)


def _table(data):
    import pyarrow as pa
    if isinstance(data, pa.Table):
        return data.combine_chunks()
    if isinstance(data, pa.RecordBatch):
        return pa.Table.from_batches([data])
    return pa.Table.from_batches(list(data)).combine_chunks()


def _blob64(arr):
    """The 64-byte blobs of a binary / large_binary / fixed_size_binary(64)
    array without nulls, as an (n, 64) uint8 array."""
    import pyarrow as pa
    n = len(arr)
    if pa.types.is_fixed_size_binary(arr.type):
        if arr.type.byte_width != 64:
            raise CudaspError(ERR_INVALID_ARG, "tweak_key must be exactly 64 bytes, got %d bytes" % arr.type.byte_width)
        data = np.frombuffer(arr.buffers()[1], dtype=np.uint8)
        return data[arr.offset * 64:(arr.offset + n) * 64].reshape(n, 64)
    ot = np.int64 if pa.types.is_large_binary(arr.type) else np.int32
    offs = np.frombuffer(arr.buffers()[1], dtype=ot)[arr.offset:arr.offset + n + 1]
    lens = np.diff(offs)
    bad = np.nonzero(lens != 64)[0]
    if bad.size:
        raise CudaspError(ERR_INVALID_ARG, "tweak_key must be exactly 64 bytes, got %d bytes" % int(lens[bad[0]]))
    data = np.frombuffer(arr.buffers()[2], dtype=np.uint8)
    return data[int(offs[0]):int(offs[0]) + 64 * n].reshape(n, 64)


def _lists(arr):
    """(per-row start offsets (n + 1, int64, from 0), int64 values) of a
    list<int64> / large_list<int64> array: a NULL list is empty, NULL elements
    are dropped (src/cudasp_extension.cu:195-221)."""
    import pyarrow as pa
    n = len(arr)
    ot = np.int64 if pa.types.is_large_list(arr.type) else np.int32
    offs = np.frombuffer(arr.buffers()[1], dtype=ot)[arr.offset:arr.offset + n + 1].astype(np.int64)
    if arr.null_count:
        valid = np.asarray(arr.is_valid())
        lens = np.where(valid, np.diff(offs), 0)
    else:
        lens = np.diff(offs)
    child = arr.values  # the whole child array (offsets index into it)
    vals = np.asarray(child.fill_null(0) if child.null_count else child).astype(np.int64, copy=False)
    starts = offs[:-1]
    # mark the child elements every (non-NULL) list covers
    cover = np.zeros(len(child) + 1, dtype=np.int64)
    np.add.at(cover, starts[lens > 0], 1)
    np.add.at(cover, (starts + lens)[lens > 0], -1)
    keep = np.cumsum(cover[:-1]) > 0
    if child.null_count:
        cvalid = np.asarray(child.is_valid())
        elem_ok = keep & cvalid
        # per-row counts of the valid elements
        pref = np.concatenate([[0], np.cumsum(elem_ok.astype(np.int64))])
        lens = pref[starts + lens] - pref[starts]
        keep = elem_ok
    out_offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return out_offs, vals[keep]


class PinnedTable:
    """A tweak table in pinned host memory, batched for the streaming scan.

        pt = PinnedTable(arrow_table)           # batch_size as cudasp_scan's (300000)
        matches = pt.scan(scan_private_key, spend_public_key, label_keys)

    batch_size as cudasp_scan's (rows per streamed batch).  devices: the GPUs
    (default [device]); batch b goes to devices[b % len(devices)], round-robin
    like the reference's threads over its GPUs (src/cudasp_extension.cu:523-529),
    each GPU with its own streaming kernel; a device listed k times runs k
    kernels on 1/k of its wave slots each (logical GPUs, as
    CUDASP_TF_DEVICE_MAP).  Holds ~64 + 8 k + 4 bytes of pinned memory per row
    (k outputs) plus a device mirror of each batch's outputs on its GPU;
    close() (or the garbage collector) frees it."""

    def __init__(self, data, batch_size=None, device=0, devices=None):
        import pyarrow as pa
        import torch
        batch_size = _batch_size_arg(batch_size)
        t = _table(data)
        if t.num_columns < 4:
            raise InvalidInputException("cudasp_scan needs the columns (txid, height, tweak_key, outputs)")
        txid, height, tweak, outputs = (t.column(i).combine_chunks() if t.column(i).num_chunks != 1
                                        else t.column(i).chunk(0) for i in range(4))
        valid = np.ones(t.num_rows, dtype=bool)
        for col in (txid, height, tweak):
            if col.null_count:
                valid &= np.asarray(col.is_valid())
        if not valid.all():
            idx = pa.array(np.nonzero(valid)[0])
            txid, height, tweak, outputs = (c.take(idx) for c in (txid, height, tweak, outputs))
        self.n = len(txid)
        self.txid, self.height = txid, height
        tw = _blob64(tweak) if self.n else np.zeros((0, 64), dtype=np.uint8)
        self.tweak = tweak
        offs, vals = _lists(outputs) if self.n else (np.zeros(1, dtype=np.int64), np.zeros(0, dtype=np.int64))
        self.devices = [int(d) for d in (devices if devices else [device])]
        self.batch_size = batch_size
        self.batches = []
        for r0 in range(0, self.n, batch_size):
            r1 = min(self.n, r0 + batch_size)
            m = r1 - r0
            o0, o1 = int(offs[r0]), int(offs[r1])
            if o1 - o0 >= 2 ** 32:
                raise CudaspError(ERR_CAPACITY, "a batch's outputs exceed u32 offsets: use a smaller batch_size")
            lg = len(self.batches) % len(self.devices)  # logical GPU of this batch
            dev = torch.device("cuda", self.devices[lg])
            b = dict(r0=r0, n=m, lg=lg)
            b["rows"] = HostBuffer(64 * m)
            b["rows"].array[:] = tw[r0:r1].reshape(-1)
            b["outputs"] = HostBuffer(max(8, 8 * (o1 - o0)))
            b["outputs"].view(np.int64)[:o1 - o0] = vals[o0:o1]
            b["offsets"] = HostBuffer(4 * (m + 1))
            b["offsets"].view(np.uint32)[:] = (offs[r0:r1 + 1] - o0).astype(np.uint32)
            b["matches"] = HostBuffer(4 * m)
            b["mirror"] = torch.empty((max(1, o1 - o0),), dtype=torch.int64, device=dev)
            self.batches.append(b)
        self.last_stats = None
        nl = len(self.devices)
        self._scanners, self._streams = [None] * nl, [None] * nl
        self._stream_ok = False
        self._stream_shape = None

    def scan(self, scan_private_key, spend_public_key, label_keys, output_count=None, label_negation=None):
        """cudasp_scan over the pinned table with these keys: every batch
        published in place to one streaming kernel (at most 64 in flight),
        then the matching rows gathered.  Returns a pyarrow Table (txid,
        height, tweak_key); last_stats gets the scan's timing."""
        import pyarrow as pa
        bound = BoundScan(scan_private_key, spend_public_key, label_keys, self.batch_size,
                          output_count=output_count, label_negation=label_negation)
        del bound  # the reference's argument checks and errors
        t0 = time.perf_counter()
        hits = []

        def collect(st, b, q):
            # a done batch's matches: its count is readable until 64 more
            # batches are published, its row indices stay in its buffer
            st.wait(q)
            c = st.matches(q)
            if c:
                hits.append(b["r0"] + b["matches"].view(np.uint32)[:c].astype(np.int64))

        # one scanner and stream per logical GPU, kept and rebound to each
        # scan's keys (a scanner's creation, its stream's and their
        # allocations cost milliseconds: a 1M-row scan takes ~6 ms on the GPU)
        labels = list(label_keys)
        shape = (len(labels), output_count or 1, bool(label_negation))
        fresh = not self._stream_ok or shape != self._stream_shape
        for lg, d in enumerate(self.devices):
            if self._scanners[lg] is None:
                self._scanners[lg] = Scanner(scan_private_key, spend_public_key, labels,
                                             max_rows=max(1, min(self.batch_size, 300000)), device=d)
            else:
                self._scanners[lg].set_keys(scan_private_key, spend_public_key, labels)
            self._scanners[lg].set_options(output_count=output_count or 1, label_negation=bool(label_negation))
            # a stream is sized (scratch, grid) for its scanner's label count
            # and output indices when created: a new one when they change
            if fresh or self._streams[lg] is None:
                if self._streams[lg] is not None:
                    self._streams[lg].close()
                self._streams[lg] = ScanStream(self._scanners[lg], self._blocks(d))
        self._stream_shape = shape
        self._stream_ok = False  # until this scan finishes
        import torch
        seqs = [[] for _ in self.devices]  # per logical GPU: (batch index, seq) in publish order
        for i, b in enumerate(self.batches):
            lg, st = b["lg"], self._streams[b["lg"]]
            with torch.cuda.device(self.devices[lg]):  # (the library sets it too; cheap insurance)
                if len(seqs[lg]) >= STREAM_RING:
                    j, q = seqs[lg][-STREAM_RING]
                    collect(st, self.batches[j], q)
                seqs[lg].append((i, st.publish(b["rows"], b["outputs"], b["offsets"], None, b["n"], None,
                                               b["mirror"], b["matches"])))
        for lg, st in enumerate(self._streams):
            with torch.cuda.device(self.devices[lg]):
                st.close_input()
        t_pub = time.perf_counter()
        for lg, st in enumerate(self._streams):
            with torch.cuda.device(self.devices[lg]):
                for j, q in seqs[lg][-STREAM_RING:]:
                    collect(st, self.batches[j], q)
                st.finish()  # the stream is reset for the next scan
        self._stream_ok = True
        idx = np.sort(np.concatenate(hits)) if hits else np.zeros(0, dtype=np.int64)
        t1 = time.perf_counter()
        ia = pa.array(idx, type=pa.int64())
        out = pa.table({"txid": self.txid.take(ia).cast(pa.binary()), "height": self.height.take(ia),
                        "tweak_key": self.tweak.take(ia).cast(pa.binary())})
        self.last_stats = dict(rows=self.n, batches=len(self.batches), matches=int(idx.size),
                               scan_s=t1 - t0, publish_s=t_pub - t0, tx_per_s=self.n / (t1 - t0) if t1 > t0 else 0.0)
        return out

    def _blocks(self, d):
        """A logical GPU's grid: its device's wave slots shared by the logical
        GPUs on it (0 = the whole device)."""
        k = self.devices.count(d)
        if k == 1:
            return 0
        import torch
        return torch.cuda.get_device_properties(d).multi_processor_count * 3 // k

    def close(self):
        for lg in range(len(self.devices)):
            if self._streams[lg] is not None:
                self._streams[lg].close()
                self._streams[lg] = None
            if self._scanners[lg] is not None:
                self._scanners[lg].close()
                self._scanners[lg] = None
        for b in self.batches:
            for k in ("rows", "outputs", "offsets", "matches"):
                b[k].close()
        self.batches = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _batch_size_arg(batch_size):
    """The bind's batch_size rules and messages (CudaspScanBind :474-487)."""
    if batch_size is None:
        return 300000
    if not isinstance(batch_size, int) or isinstance(batch_size, bool):
        raise InvalidInputException("batch_size parameter must be an INTEGER")
    if batch_size <= 0:
        raise InvalidInputException("batch_size must be positive, got %d" % batch_size)
    if batch_size > 10_000_000:
        raise InvalidInputException("batch_size too large (max 10,000,000), got %d" % batch_size)
    return batch_size


class NativePinnedTable:
    """PinnedTable on the C pinned-table ABI (include/cudasp_host.h,
    cudasp_pinned_*; csrc/host/pinned_table.cpp): the rows reach pinned memory
    through cudasp_pinned_append (Arrow buffers, bulk reads, the
    table-function host's row semantics) and each scan's publish / harvest
    loop runs in C++.  Same constructor, scan(), last_stats and close() as
    PinnedTable; what a DuckDB host would call beside cudasp_scan.
    placement="hbm" keeps the table resident in device memory instead
    (CUDASP_TABLE_HBM: each scan one k_scan_multi launch per GPU over all of
    its batches)."""

    PLACEMENTS = {"pinned": 0, "hbm": 1}  # CUDASP_TABLE_PINNED / CUDASP_TABLE_HBM

    def __init__(self, data, batch_size=None, device=0, devices=None, piece_rows=1 << 20, placement="pinned"):
        import ctypes

        from . import _native
        from .table_function import _arrow_pieces, _columns, _lib
        self.batch_size = _batch_size_arg(batch_size)
        t = _table(data)
        if t.num_columns < 4:
            raise InvalidInputException("cudasp_scan needs the columns (txid, height, tweak_key, outputs)")
        self.txid, self.height, self.tweak = (t.column(i).combine_chunks() if t.column(i).num_chunks != 1
                                              else t.column(i).chunk(0) for i in range(3))
        self.n = t.num_rows
        self.devices = [int(d) for d in (devices if devices else [device])]
        lib = self._lib = _lib()
        h = ctypes.c_void_p()
        devs = (ctypes.c_int * len(self.devices))(*self.devices)
        if placement not in self.PLACEMENTS:
            raise ValueError("placement must be 'pinned' or 'hbm', got %r" % (placement,))
        _native.check(lib.cudasp_pinned_create_placed(self.batch_size, devs, len(self.devices),
                                                      self.PLACEMENTS[placement], ctypes.byref(h)))
        self._h = h
        try:
            for piece in _arrow_pieces(t, piece_rows):  # row numbers: positions in t
                cols = _columns(*piece)
                _native.check(lib.cudasp_pinned_append(h, ctypes.byref(cols)))
        except Exception:
            self.close()
            raise
        self.last_stats = None

    def info(self):
        import ctypes

        from . import _native
        from .table_function import _PinnedInfo
        st = _PinnedInfo()
        _native.check(self._lib.cudasp_pinned_info(self._h, ctypes.byref(st)))
        return {name: getattr(st, name) for name, _ in _PinnedInfo._fields_}

    def scan_rows(self, scan_private_key, spend_public_key, label_keys, output_count=None, label_negation=None):
        """The matching rows' numbers (positions in the table), ascending."""
        import ctypes

        from . import _native
        bound = BoundScan(scan_private_key, spend_public_key, label_keys, self.batch_size,
                          output_count=output_count, label_negation=label_negation)
        rows = ctypes.POINTER(ctypes.c_uint64)()
        count = ctypes.c_uint64()
        _native.check(self._lib.cudasp_pinned_scan(self._h, bound._h, ctypes.byref(rows), ctypes.byref(count)))
        try:
            idx = np.ctypeslib.as_array(rows, (count.value,)).astype(np.int64) if count.value else \
                np.zeros(0, dtype=np.int64)
        finally:
            self._lib.cudasp_pinned_free_rows(rows)
        return idx

    def scan(self, scan_private_key, spend_public_key, label_keys, output_count=None, label_negation=None):
        """As PinnedTable.scan: a pyarrow Table (txid, height, tweak_key)."""
        import pyarrow as pa
        t0 = time.perf_counter()
        idx = self.scan_rows(scan_private_key, spend_public_key, label_keys, output_count, label_negation)
        t1 = time.perf_counter()
        ia = pa.array(idx, type=pa.int64())
        out = pa.table({"txid": self.txid.take(ia).cast(pa.binary()), "height": self.height.take(ia),
                        "tweak_key": self.tweak.take(ia).cast(pa.binary())})
        inf = self.info()
        self.last_stats = dict(rows=self.n, batches=inf["batches"], matches=int(idx.size), scan_s=t1 - t0,
                               native_scan_s=inf["last_scan_s"], publish_s=inf["last_publish_s"],
                               tx_per_s=self.n / (t1 - t0) if t1 > t0 else 0.0)
        return out

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.cudasp_pinned_free(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
