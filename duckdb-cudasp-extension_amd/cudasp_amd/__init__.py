"""cudasp_amd -- MI355X-native cudasp_scan (BIP-352 silent-payment scanning).

The compute path is the HIP library ``libcudasp_amd.so`` (gfx950 kernels behind
the C ABI in ``include/cudasp_abi.h``, table-function host behind
``include/cudasp_host.h``); this package is its Python face.
"""
from ._native import CudaspError, load as load_native  # noqa: F401
from .scanner import HostBuffer, Scanner, ScanStream, StreamBatch  # noqa: F401
from .pinned import NativePinnedTable, PinnedTable  # noqa: F401
from .table_function import (BoundScan, assign_gpu, InvalidInputException, cudasp_scan, cudasp_scan_arrow, pool_size,  # noqa: F401
                             prewarm, release_pool)
