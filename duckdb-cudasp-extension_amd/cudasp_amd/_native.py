"""ctypes binding of the in-tree HIP library ``libcudasp_amd.so``.

The library is the product: every compute call goes to the gfx950 kernels
through the C ABI declared in ``include/cudasp_abi.h``.  There is no CPU
fallback; if the library is missing or no device is visible, calls raise.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "libcudasp_amd.so")

CUDASP_OK = 0
CUDASP_ERR_INVALID_ARG = -2
CUDASP_ERR_HIP = -3
CUDASP_ERR_NO_DEVICE = -4
CUDASP_ERR_CAPACITY = -5

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_I32 = ctypes.c_int

# name -> (restype, argtypes); mirrors include/cudasp_abi.h
SIGNATURES = {
    "cudasp_last_error": (ctypes.c_char_p, []),
    "cudasp_version": (ctypes.c_char_p, []),
    "cudasp_device_count": (_I32, []),
    "cudasp_scanner_create": (_I32, [_I32, _P, _P, _P, _U32, _U32, ctypes.POINTER(_P)]),
    "cudasp_scanner_destroy": (None, [_P]),
    "cudasp_scanner_set_keys": (_I32, [_P, _P, _P, _P, _U32]),
    "cudasp_scanner_set_options": (_I32, [_P, _P]),
    "cudasp_default_fixed_base_bits": (_I32, []),
    "cudasp_fixed_base_table_bytes": (ctypes.c_uint64, [_I32]),
    "cudasp_scanner_set_fixed_base_bits": (_I32, [_P, _I32]),
    "cudasp_fixed_base_prepare": (_I32, [_I32, _I32, ctypes.POINTER(ctypes.c_double)]),
    "cudasp_debug_fb_check": (_I32, [_I32, _I32, _U32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "cudasp_debug_fold_check": (_I32, [_I32, _I32, ctypes.c_char_p, _U32, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_uint64)]),
    "cudasp_scanner_fixed_base_bits": (_I32, [_P]),
    "cudasp_scanner_set_spend_fold": (_I32, [_P, _I32]),
    "cudasp_scanner_spend_folded": (_I32, [_P]),
    "cudasp_scanner_set_rows_per_thread": (_I32, [_P, _I32, _I32]),
    "cudasp_scan_device": (_I32, [_P, _P, _P, _P, _P, _P, _U32, _P, _P, _P, _P]),
    "cudasp_scan_host": (_I32, [_P, _P, _P, ctypes.c_size_t, _P, _P, _U32, _P]),
    "cudasp_row_values_device": (_I32, [_P, _P, _P, _U32, _P, _P, _P]),
    "cudasp_scan_device_batches": (_I32, [_P, _P, _U32, _P]),
    "cudasp_scanner_sync": (_I32, [_P]),
    "cudasp_tweaks_to_columns": (_I32, [_P, _U32, _P, _P, _P]),
    "cudasp_stage_shared_secret_device": (_I32, [_P, _P, _P, _U32, _P, _P]),
    "cudasp_stage_match_device": (_I32, [_P, _P, _P, _P, _P, _U32, _P, _P, _P, _P]),
    "cudasp_layout_probe": (_I32, [_P, _P, _U32, _P, _P, _P, _P, _P]),
    "cudasp_synth_tweak_columns": (_I32, [_I32, _P, ctypes.c_uint64, _U32, _P, _P, _P]),
    "cudasp_synth_outputs": (_I32, [ctypes.c_uint64, ctypes.c_uint64, _U32, _U32, _P, _P, _P, _P]),
    "cudasp_synth_output_lengths": (_I32, [ctypes.c_uint64, ctypes.c_uint64, _U32, _U32, _P, _P]),
    "cudasp_synth_output_values": (_I32, [ctypes.c_uint64, ctypes.c_uint64, _U32, _P, _P, _P, _P]),
    "cudasp_host_alloc": (_I32, [ctypes.POINTER(_P), ctypes.c_size_t]),
    "cudasp_host_free": (None, [_P]),
    "cudasp_stream_supported": (_I32, [_P]),
    "cudasp_stream_create": (_I32, [_P, _U32, ctypes.POINTER(_P)]),
    "cudasp_stream_publish": (_I32, [_P, _P, _P, _P, _P, _U32, _P, _P, ctypes.POINTER(ctypes.c_uint64)]),
    "cudasp_stream_publish_batch": (_I32, [_P, _P, ctypes.POINTER(ctypes.c_uint64)]),
    "cudasp_stream_close": (_I32, [_P]),
    "cudasp_stream_query": (_I32, [_P, ctypes.c_uint64]),
    "cudasp_stream_wait": (_I32, [_P, ctypes.c_uint64]),
    "cudasp_stream_set_timeout": (_I32, [_P, _U32]),
    "cudasp_stream_matches": (_I32, [_P, ctypes.c_uint64, ctypes.POINTER(_U32)]),
    "cudasp_stream_finish": (_I32, [_P]),
    "cudasp_stream_abandoned": (_I32, [_P]),
    "cudasp_stream_stats": (_I32, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(_U32)]),
    "cudasp_stream_counters": (_I32, [_P, ctypes.POINTER(ctypes.c_uint64), _U32]),
    "cudasp_stream_destroy": (None, [_P]),
    "cudasp_debug_field_ops": (_I32, [ctypes.c_int, _P, _P, _P, _U32]),
    "cudasp_field_layout": (_I32, [_P, _P, _P, _P, _P]),
    "LaunchBatchScan": (_P, [_P, _P, _P, _P, _P, _P, _P, _U32, _P, _P, _P, _P, _U32, ctypes.c_size_t]),
    "RunBatchScanKernels": (_I32, [_P, _P, _P, _P, _P, _P, _P, _P, _U32, _P, _U32]),
    "FreeBatchScanState": (None, [_P]),
    "FreeBatchScanManaged": (None, [_P]),
}


class CudaspError(RuntimeError):
    def __init__(self, code, message):
        super().__init__("cudasp error %d: %s" % (code, message))
        self.code = code


_lib = None


def load(path=None):
    """Load (once) and return the native library; raises if it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("CUDASP_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise CudaspError(CUDASP_ERR_NO_DEVICE,
                          "HIP library %s not built (run `make -C duckdb-cudasp-extension_amd` "
                          "or __graft_entry__.build())" % p)
    # No import order to keep: the library names the HIP runtime by the file
    # name torch's libraries use (DT_NEEDED libamdhip64.so, see the Makefile),
    # so it and torch share one runtime whichever loads first
    # (tools/probes/init_order.py, tests/test_init_order_gpu.py).
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(rc):
    if rc != CUDASP_OK:
        msg = load().cudasp_last_error()
        raise CudaspError(rc, msg.decode() if msg else "")
    return rc


CUDASP_STREAM_DEFAULT = 1  # include/cudasp_abi.h: the device's null stream
CUDASP_MAX_OUTPUT_COUNT = 64


class DeviceBatch(ctypes.Structure):
    """cudasp_device_batch (include/cudasp_abi.h)."""
    _fields_ = [("tweak_x", _P), ("tweak_y", _P), ("outputs", _P), ("output_offsets", _P),
                ("output_lengths", _P), ("n", _U32), ("match_flags", _P), ("match_rows", _P),
                ("match_count", _P)]


class StreamBatchDesc(ctypes.Structure):
    """cudasp_stream_batch (include/cudasp_abi.h)."""
    _fields_ = [("tweak_keys", _P), ("outputs", _P), ("output_offsets", _P), ("output_lengths", _P),
                ("n", _U32), ("match_flags", _P), ("match_rows", _P), ("d_mirror", _P)]


class ScanOptions(ctypes.Structure):
    """cudasp_scan_options (include/cudasp_abi.h)."""
    _fields_ = [("output_count", ctypes.c_uint32), ("label_negation", ctypes.c_uint32),
                ("full_x", ctypes.c_uint32)]


def stream_arg(stream):
    """A torch stream as the ABI's `stream` argument.  torch's default stream
    has handle 0, which the ABI reads as "the scanner's own stream"; it is
    passed as CUDASP_STREAM_DEFAULT so the launch stays ordered with the work
    torch queued on it."""
    h = stream.cuda_stream
    return ctypes.c_void_p(h if h else CUDASP_STREAM_DEFAULT)
