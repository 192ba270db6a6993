"""Device data-plane operators (HIP kernels for gfx950, NumPy for CPU tensors)."""
from .primitives import (HashTable, tokenize, key_meta, key_bytes_list, exclusive_scan, gather_key_bytes,  # noqa: F401
                         copy_to_host, host_read, host_read_many, host_read_begin,
                         sort_keys, sort_keys_checked, sort_error, debug_sort_fail, sort_by_partition_key, bincount, reduce_by_key, next_pow2,
                         exact_key_perm, gather_aos4)
from . import keys  # noqa: F401
