"""Scanner: one query's keys bound on one MI355X device.

Thin Python face of ``cudasp_scanner_*`` (include/cudasp_abi.h).  Device
buffers are torch tensors (PyTorch is only the allocator / stream provider
here); host buffers are numpy arrays.  The device-path methods run on `stream`
or, when it is None, on torch's current stream of the scanner's device (so
they are ordered after the torch work that produced their inputs, as any torch
op would be); sync() waits for both that stream and the scanner's own.
"""
import ctypes

import numpy as np

from . import _native


class DeviceBatches:
    """A prepared cudasp_device_batch array (Scanner.device_batches): the
    descriptors of include/cudasp_abi.h, plus references that keep the
    tensors they point into alive."""

    def __init__(self, batches):
        batches = list(batches)
        self.count = len(batches)
        self.array = (_native.DeviceBatch * max(1, self.count))()
        for i, b in enumerate(batches):
            self.array[i] = _native.DeviceBatch(
                _ptr(b["tweak_x"]), _ptr(b["tweak_y"]), _ptr(b.get("outputs")), _ptr(b["offsets"]),
                _ptr(b["lengths"]), int(b["flags"].numel()), _ptr(b["flags"]), _ptr(b.get("match_rows")),
                _ptr(b.get("match_count")))
        self._refs = batches


def _ptr(t):
    """Raw pointer of a torch tensor or numpy array (None -> NULL)."""
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return t.ctypes.data
    return t.data_ptr()


def _as_bytes(b, n, what):
    if isinstance(b, (bytes, bytearray)):
        if len(b) != n:
            raise ValueError("%s must be exactly %d bytes, got %d bytes" % (what, n, len(b)))
        return bytes(b)
    raise TypeError("%s must be bytes" % what)


class Scanner:
    """Bind scan key, spend key and label keys on `device` for batches of at
    most `max_rows` rows (CudaspScanBindData + LaunchBatchScan of the
    reference, src/cudasp_extension.cu:87-104, src/cudasp_gpu.cu:445-669)."""

    def __init__(self, scan_private_key, spend_public_key, label_keys=(), max_rows=300000, device=0):
        lib = _native.load()
        scan = _as_bytes(scan_private_key, 32, "scan_private_key")
        spend = _as_bytes(spend_public_key, 64, "spend_public_key")
        labels = [_as_bytes(l, 64, "label key") for l in label_keys]
        self.label_count = len(labels)
        self.max_rows = int(max_rows)
        self.device = int(device)
        lab = b"".join(labels) if labels else None
        h = ctypes.c_void_p()
        _native.check(lib.cudasp_scanner_create(self.device, scan, spend, lab, self.label_count,
                                                self.max_rows, ctypes.byref(h)))
        self._h = h
        self._lib = lib
        self.output_count = 1
        self.label_negation = False
        self.full_x = False

    def set_options(self, output_count=1, label_negation=False, full_x=False):
        """Protocol variants (cudasp_scanner_set_options):
        output indices k = 0..output_count-1, labels also negated, outputs as
        32-byte big-endian x-only keys compared in full.  The defaults are the
        reference's semantics."""
        opt = _native.ScanOptions(int(output_count), int(bool(label_negation)), int(bool(full_x)))
        _native.check(self._lib.cudasp_scanner_set_options(self._h, ctypes.byref(opt)))
        self.output_count = int(output_count)
        self.label_negation = bool(label_negation)
        self.full_x = bool(full_x)
        self._t = None

    def set_fixed_base_bits(self, bits=0):
        """Fixed-base window width of stage B (22 or 26; 0 = the process
        default, cudasp_default_fixed_base_bits).  Same results at every
        width; builds the device's table for that width on first use."""
        _native.check(self._lib.cudasp_scanner_set_fixed_base_bits(self._h, int(bits)))

    def set_spend_fold(self, on=True):
        """The spend key folded into the fixed-base table's top window
        (cudasp_scanner_set_spend_fold; on by default for an on-curve key at an
        HBM width).  Same results either way."""
        _native.check(self._lib.cudasp_scanner_set_spend_fold(self._h, int(bool(on))))

    @property
    def spend_folded(self):
        """Whether this scanner's launches use the folded top window."""
        return bool(self._lib.cudasp_scanner_spend_folded(self._h))

    def set_rows_per_thread(self, rows_a=0, rows_b=0):
        """Launch shape of the next launches (cudasp_scanner_set_rows_per_thread):
        rows per thread of stage A (1, 2, 4) and stage B (2, 6); 0 = automatic."""
        _native.check(self._lib.cudasp_scanner_set_rows_per_thread(self._h, int(rows_a), int(rows_b)))

    @property
    def fixed_base_bits(self):
        return int(self._lib.cudasp_scanner_fixed_base_bits(self._h))

    @property
    def value_rows(self):
        """Compare values per virtual row: the base value and one per label
        (labels twice with label_negation)."""
        return 1 + (2 if self.label_negation else 1) * self.label_count

    def set_keys(self, scan_private_key, spend_public_key, label_keys=()):
        """Rebind to another query's keys, keeping the device buffers
        (cudasp_scanner_set_keys)."""
        scan = _as_bytes(scan_private_key, 32, "scan_private_key")
        spend = _as_bytes(spend_public_key, 64, "spend_public_key")
        labels = [_as_bytes(l, 64, "label key") for l in label_keys]
        lab = b"".join(labels) if labels else None
        _native.check(self._lib.cudasp_scanner_set_keys(self._h, scan, spend, lab, len(labels)))
        self.label_count = len(labels)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.cudasp_scanner_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ----------------------------------------------------------- device path
    def _stream(self, stream):
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(torch.device("cuda", self.device))
        return _native.stream_arg(stream)

    def scan_device(self, tweak_x, tweak_y, outputs, offsets, lengths, flags, match_rows=None,
                    match_count=None, stream=None):
        """Asynchronous scan of device-resident columns (torch tensors)."""
        n = int(flags.numel())
        st = self._stream(stream)
        _native.check(self._lib.cudasp_scan_device(
            self._h, _ptr(tweak_x), _ptr(tweak_y), _ptr(outputs), _ptr(offsets), _ptr(lengths), n,
            _ptr(flags), _ptr(match_rows), _ptr(match_count), st))

    def scan_device_batches(self, batches, stream=None):
        """Asynchronous scan of several device-resident batches in one call
        (cudasp_scan_device_batches: one persistent kernel for both stages).
        batches: sequence of dicts with the keys of scan_device (tweak_x,
        tweak_y, outputs, offsets, lengths, flags, optional match_rows /
        match_count); n is flags.numel().  Or the DeviceBatches of
        device_batches(...), for a set scanned repeatedly: the C array is then
        built once, not on every call."""
        if not isinstance(batches, DeviceBatches):
            batches = DeviceBatches(batches)
        st = self._stream(stream)
        _native.check(self._lib.cudasp_scan_device_batches(self._h, batches.array, batches.count, st))

    @staticmethod
    def device_batches(batches):
        """The cudasp_device_batch array of `batches` (as for
        scan_device_batches), built once; it holds references to the tensors."""
        return DeviceBatches(batches)

    def row_values_device(self, tweak_x, tweak_y, t_out, values, stream=None):
        n = int(tweak_x.numel() // 8)
        st = self._stream(stream)
        _native.check(self._lib.cudasp_row_values_device(
            self._h, _ptr(tweak_x), _ptr(tweak_y), n, _ptr(t_out), _ptr(values), st))

    def stage_shared_secret(self, tweak_x, tweak_y, n, stream=None, t_out=None):
        """Launch only stage A (d*T, serialize, tagged hash) for n rows; t goes to
        t_out or to a scanner-held buffer used by the next stage_match."""
        if t_out is None:
            import torch
            if getattr(self, "_t", None) is None:
                self._t = torch.empty((8 * self.max_rows * self.output_count,), dtype=torch.int32,
                                      device=torch.device("cuda", self.device))
            t_out = self._t
        self._t_last = t_out
        st = self._stream(stream)
        _native.check(self._lib.cudasp_stage_shared_secret_device(
            self._h, _ptr(tweak_x), _ptr(tweak_y), int(n), _ptr(t_out), st))

    def stage_match(self, outputs, offsets, lengths, n, flags, match_rows=None, match_count=None, stream=None,
                    t_in=None):
        """Launch only stage B on the t of the previous stage_shared_secret."""
        t_in = self._t_last if t_in is None else t_in
        st = self._stream(stream)
        _native.check(self._lib.cudasp_stage_match_device(
            self._h, _ptr(t_in), _ptr(outputs), _ptr(offsets), _ptr(lengths), int(n), _ptr(flags),
            _ptr(match_rows), _ptr(match_count), st))

    def sync(self):
        import torch
        torch.cuda.current_stream(torch.device("cuda", self.device)).synchronize()
        _native.check(self._lib.cudasp_scanner_sync(self._h))

    # ------------------------------------------------------------- host path
    def scan_host(self, tweak_keys, outputs, offsets, lengths):
        """Synchronous scan from host memory.  tweak_keys: uint8 [n, 64];
        outputs: int64 CSR values (with full_x: uint8 [total, 32] big-endian
        x-only keys); offsets/lengths: uint32 [n], counting outputs.  Returns a
        uint8 [n] array of match flags."""
        tk = np.ascontiguousarray(tweak_keys, dtype=np.uint8).reshape(-1, 64)
        n = tk.shape[0]
        if self.full_x:
            outs = np.ascontiguousarray(outputs, dtype=np.uint8).reshape(-1, 32)
        else:
            outs = np.ascontiguousarray(outputs, dtype=np.int64)
        offs = np.ascontiguousarray(offsets, dtype=np.uint32)
        lens = np.ascontiguousarray(lengths, dtype=np.uint32)
        if offs.shape[0] != n or lens.shape[0] != n:
            raise ValueError("offsets/lengths must have one entry per row")
        flags = np.zeros(n, dtype=np.uint8)
        if n == 0:
            return flags
        _native.check(self._lib.cudasp_scan_host(
            self._h, _ptr(tk), _ptr(outs) if outs.size else None, outs.shape[0], _ptr(offs), _ptr(lens), n,
            _ptr(flags)))
        return flags


# ------------------------------------------------------------- streaming scan
class HostBuffer:
    """Coherent pinned host memory (cudasp_host_alloc), device-addressable at
    the same address: what a streamed batch's host buffers must live in.
    ``array`` is a uint8 numpy view; ``view(dtype)`` reinterprets it."""

    def __init__(self, nbytes):
        self._lib = _native.load()
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        _native.check(self._lib.cudasp_host_alloc(ctypes.byref(p), max(1, self.nbytes)))
        self.ptr = p.value
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, self.nbytes)).from_address(self.ptr))

    def view(self, dtype):
        return self.array.view(dtype)

    def close(self):
        if getattr(self, "ptr", None):
            self.array = None
            self._lib.cudasp_host_free(ctypes.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ScanStream:
    """cudasp_stream_*: ONE persistent kernel scans the batches published
    into it, reading them from pinned host memory (HostBuffer) and writing
    their flags back there (include/cudasp_abi.h).  The scanner must not run
    other launches while the stream is open."""

    def __init__(self, scanner, blocks=0):
        self._lib = _native.load()
        self.scanner = scanner
        h = ctypes.c_void_p()
        _native.check(self._lib.cudasp_stream_create(scanner._h, int(blocks), ctypes.byref(h)))
        self._h = h

    def publish(self, rows, outputs, offsets, lengths, n, flags, mirror=None, matches=None):
        """rows / outputs / offsets / lengths / flags / matches: HostBuffers
        (or their addresses; flags or matches may be None) that the kernel
        reads and writes in place; mirror: a device tensor of the batch's
        outputs size.  Returns the batch's sequence number."""
        seq = ctypes.c_uint64()
        addr = lambda b: None if b is None else (b.ptr if isinstance(b, HostBuffer) else int(b))  # noqa: E731
        d = _native.StreamBatchDesc(addr(rows), addr(outputs), addr(offsets), addr(lengths), int(n), addr(flags),
                                    addr(matches), None if mirror is None else mirror.data_ptr())
        _native.check(self._lib.cudasp_stream_publish_batch(self._h, ctypes.byref(d), ctypes.byref(seq)))
        return seq.value

    def close_input(self):
        """No batch follows (cudasp_stream_close): the kernel ends once the
        published batches are done."""
        _native.check(self._lib.cudasp_stream_close(self._h))

    def query(self, seq):
        rc = self._lib.cudasp_stream_query(self._h, int(seq))
        if rc < 0:
            _native.check(rc)
        return rc == 1

    def wait(self, seq):
        _native.check(self._lib.cudasp_stream_wait(self._h, int(seq)))

    def set_timeout(self, ms):
        _native.check(self._lib.cudasp_stream_set_timeout(self._h, int(ms)))

    def matches(self, seq):
        """Matching rows of done batch `seq` (cudasp_stream_matches)."""
        c = ctypes.c_uint32()
        _native.check(self._lib.cudasp_stream_matches(self._h, int(seq), ctypes.byref(c)))
        return c.value

    def abandoned(self):
        return bool(self._lib.cudasp_stream_abandoned(self._h))

    def finish(self):
        _native.check(self._lib.cudasp_stream_finish(self._h))

    def stats(self):
        launches, blocks = ctypes.c_uint64(), ctypes.c_uint32()
        _native.check(self._lib.cudasp_stream_stats(self._h, ctypes.byref(launches), ctypes.byref(blocks)))
        return {"launches": launches.value, "blocks": blocks.value}

    COUNTERS = ("pieces", "wave_rows", "wait_polls", "drains", "reserved", "worker_exits", "idle_exits",
                "poller_polls", "busy_ticks", "life_ticks")

    def counters(self):
        """The kernel's counters of the last finished query (cudasp_stream_counters)."""
        v = (ctypes.c_uint64 * 16)()
        _native.check(self._lib.cudasp_stream_counters(self._h, v, 16))
        return dict(zip(self.COUNTERS, list(v)))

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.cudasp_stream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class StreamBatch:
    """One batch staged in pinned host memory for a ScanStream: the tweak
    blobs, the outputs CSR (int64 values, or 32-byte keys with full_x), the
    flags and the match indices the kernel writes, and the device mirror of
    the outputs the kernel's compares read."""

    def __init__(self, tweak_keys, outputs, offsets, lengths, label_count=0, device=0, full_x=False,
                 want_flags=True, want_matches=True):
        tk = np.ascontiguousarray(tweak_keys, dtype=np.uint8).reshape(-1, 64)
        self.n = tk.shape[0]
        outs = (np.ascontiguousarray(outputs, dtype=np.uint8).reshape(-1) if full_x
                else np.ascontiguousarray(outputs, dtype=np.int64).view(np.uint8).reshape(-1))
        self.rows = HostBuffer(tk.nbytes)
        self.rows.array[:] = tk.reshape(-1)
        self.outputs = HostBuffer(max(8, outs.nbytes))
        self.outputs.array[:outs.nbytes] = outs
        self.offsets = HostBuffer(4 * self.n)
        self.offsets.view(np.uint32)[:] = np.asarray(offsets, dtype=np.uint32)
        self.lengths = HostBuffer(4 * self.n)
        self.lengths.view(np.uint32)[:] = np.asarray(lengths, dtype=np.uint32)
        self.flags = HostBuffer(self.n) if want_flags else None
        if self.flags is not None:
            self.flags.array[:] = 0xEE  # every row must be written
        self.match_rows = HostBuffer(4 * max(1, self.n)) if want_matches else None
        import torch
        dev = torch.device("cuda", device)
        self.mirror = torch.empty((max(1, outs.nbytes // 8),), dtype=torch.int64, device=dev)
        self.output_words = outs.nbytes // 8
        self.seq = None

    def publish(self, stream):
        self.seq = stream.publish(self.rows, self.outputs, self.offsets, self.lengths, self.n, self.flags,
                                  self.mirror, self.match_rows)
        return self.seq

    def refill(self, tweak_keys, outputs, offsets, lengths):
        """Another batch into the same pinned buffers and device mirror (a
        host's slot reused once its previous batch is done): at most the rows
        and output bytes the buffers were made for (int64 outputs)."""
        tk = np.ascontiguousarray(tweak_keys, dtype=np.uint8).reshape(-1)
        outs = np.ascontiguousarray(outputs, dtype=np.int64).view(np.uint8).reshape(-1)
        n = tk.size // 64
        if n == 0 or tk.size > self.rows.nbytes or outs.nbytes > self.outputs.nbytes or 4 * n > self.offsets.nbytes:
            raise ValueError("refill: %d rows / %d output bytes exceed the batch's buffers" % (n, outs.nbytes))
        self.rows.array[:tk.size] = tk
        self.outputs.array[:outs.nbytes] = outs
        self.offsets.view(np.uint32)[:n] = np.asarray(offsets, dtype=np.uint32)
        self.lengths.view(np.uint32)[:n] = np.asarray(lengths, dtype=np.uint32)
        self.n = n
        self.output_words = outs.nbytes // 8
        self.reset()

    def reset(self):
        if self.flags is not None:
            self.flags.array[:] = 0xEE
        if self.match_rows is not None:
            self.match_rows.array[:] = 0xEE

    def result(self):
        return self.flags.array[:self.n].copy()

    def matches(self, stream):
        """The matching rows (sorted) of this batch once it is done."""
        c = stream.matches(self.seq)
        return np.sort(self.match_rows.view(np.uint32)[:c].copy())
