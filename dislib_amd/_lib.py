"""ctypes binding of ``libdkm.so`` (the C ABI declared in ``include/dkm.h``).

The product path has no CPU fallback: if the HIP library is missing or no
GPU is visible, :func:`lib` raises.  Symbols are resolved eagerly so that a
stale or partial build fails at load time, not mid-fit.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DKM_LIB", os.path.join(_HERE, "libdkm.so"))

# constants mirrored from include/dkm.h
ABI_VERSION = 3
MODE_AUTO, MODE_EXACT, MODE_SCREEN32, MODE_BF16X3, MODE_BF16 = 0, 1, 2, 3, 4
MODE_MASK, MODE_NOHINT, MODE_B1, MODE_TRANSLATE = 0xff, 0x100, 0x200, 0x400
IMAGE_NONE, IMAGE_SINGLE, IMAGE_SPLIT, IMAGE_SORTED, IMAGE_GEMM = 0, 1, 2, 3, 4
IMAGE_BUILD = 0x100   # kind flag: build the allocated image during the call
SUMS_F64, SUMS_F32, SUMS_RECIP = 0, 1, 2
PREP_CSR = 1
COMM_ID_BYTES = 128

_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_sz = ctypes.c_size_t
_f64 = ctypes.c_double
_u64 = ctypes.c_uint64

# name -> (restype, argtypes): every entry point of include/dkm.h
SIGNATURES = {
    "dkm_abi_version": (_i32, []),
    "dkm_preload": (_i32, []),
    "dkm_last_error": (ctypes.c_char_p, []),
    "dkm_workspace_bytes": (_sz, [_i64, _i64, _i64]),
    "dkm_prepare_centers": (_i32, [_p, _i64, _i64, _i32, _p, _sz, _p, _p]),
    "dkm_partial_sum_f64": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _p, _sz,
                                   _p, _p, _i32, _p]),
    "dkm_partial_sum_f32": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _p, _sz,
                                   _p, _p, _i32, _p]),
    "dkm_assign_delta_f64": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _p, _sz,
                                    _p, _p, _i32, _p]),
    "dkm_assign_delta_f32": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _p, _sz,
                                    _p, _p, _i32, _p]),
    "dkm_x_image_kind": (_i32, [_i64, _i64, _i32]),
    "dkm_x_image_bytes": (_sz, [_i64, _i64, _i32]),
    "dkm_x_image_f64": (_i32, [_p, _i64, _i64, _i64, _i32, _p, _sz, _p]),
    "dkm_x_image_f32": (_i32, [_p, _i64, _i64, _i64, _i32, _p, _sz, _p]),
    "dkm_x_image_sorted_ok": (_i32, [_i64, _i64]),
    "dkm_x_image_sorted_f64": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _p,
                                      _sz, _p, _sz, _p]),
    "dkm_x_image_sorted_f32": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _p,
                                      _sz, _p, _sz, _p]),
    "dkm_x_image_sorted_sums_f64": (_i32, [_p, _i64, _i64, _i64, _p, _i64,
                                           _p, _sz, _p, _sz, _p, _p]),
    "dkm_x_image_sorted_sums_f32": (_i32, [_p, _i64, _i64, _i64, _p, _i64,
                                           _p, _sz, _p, _sz, _p, _p]),
    "dkm_partial_sum_img_f64": (_i32, [_p, _p, _i32, _sz, _i64, _i64, _i64,
                                       _p, _i64, _p, _sz, _p, _p, _i32, _p]),
    "dkm_partial_sum_img_f32": (_i32, [_p, _p, _i32, _sz, _i64, _i64, _i64,
                                       _p, _i64, _p, _sz, _p, _p, _i32, _p]),
    "dkm_assign_delta_img_f64": (_i32, [_p, _p, _i32, _sz, _i64, _i64, _i64,
                                        _p, _i64, _p, _sz, _p, _p, _i32, _p]),
    "dkm_assign_delta_img_f32": (_i32, [_p, _p, _i32, _sz, _i64, _i64, _i64,
                                        _p, _i64, _p, _sz, _p, _p, _i32, _p]),
    "dkm_label_sums_f64": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _p, _sz,
                                  _p, _p]),
    "dkm_label_sums_f32": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _p, _sz,
                                  _p, _p]),
    "dkm_add_f64": (_i32, [_p, _p, _i64, _p]),
    "dkm_add_f64_nz": (_i32, [_p, _p, _i64, _p, _p]),
    "dkm_add_f64_dd": (_i32, [_p, _p, _p, _i64, _p, _p]),
    "dkm_predict_f64": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _p, _sz, _p,
                               _i32, _p]),
    "dkm_predict_f32": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _p, _sz, _p,
                               _i32, _p]),
    "dkm_update_centers": (_i32, [_p, _p, _i64, _i64, _i32, _f64, _p, _p,
                                  _p]),
    "dkm_partial_sum_csr_f64": (_i32, [_p, _p, _p, _i64, _i64, _p, _i64, _p,
                                       _sz, _p, _p, _p]),
    "dkm_assign_delta_csr_f64": (_i32, [_p, _p, _p, _i64, _i64, _p, _i64,
                                        _p, _sz, _p, _p, _p]),
    "dkm_predict_csr_f64": (_i32, [_p, _p, _p, _i64, _i64, _p, _i64, _p, _sz,
                                   _p, _p]),
    "dkm_make_blobs_f64": (_i32, [_p, _i64, _i64, _i64, _i64, _u64, _f64,
                                  _f64, _p, _p]),
    "dkm_screen_stats": (_i32, [_p, ctypes.POINTER(_i64), _p]),
    "dkm_screen_counters": (_i32, [_p, ctypes.POINTER(_i64), _p]),
    "dkm_screen_lists": (_i32, [_p, ctypes.c_size_t, ctypes.POINTER(_i64),
                                _p]),
    # distance-primitive reuse (kNN, DBSCAN epsilon query)
    "dkm_knn_workspace_bytes": (_sz, [_i64, _i64, _i64]),
    "dkm_knn_f64": (_i32, [_p, _i64, _i64, _p, _i64, _i64, _i64, _i64, _p,
                           _sz, _p, _p, _p]),
    "dkm_knn_csr_f64": (_i32, [_p, _p, _p, _i64, _p, _p, _p, _i64, _i64,
                               _i64, _i32, _p, _sz, _p, _p, _p]),
    "dkm_radius_count_f64": (_i32, [_p, _i64, _i64, _p, _i64, _i64, _i64,
                                    _f64, _p, _p]),
    "dkm_radius_workspace_bytes": (_sz, [_i64, _i64]),
    "dkm_radius_count_csr_f64": (_i32, [_p, _p, _p, _i64, _i64, _i64, _i64,
                                        _f64, _i32, _p, _p]),
    "dkm_radius_fill_csr_f64": (_i32, [_p, _p, _p, _i64, _i64, _i64, _i64,
                                       _f64, _i32, _p, _p, _sz, _p, _p, _p]),
    "dkm_radius_fill_f64": (_i32, [_p, _i64, _i64, _p, _i64, _i64, _i64,
                                   _f64, _p, _p, _sz, _p, _p, _p]),
    # multi-GPU all-reduce (RCCL)
    "dkm_allreduce_unique_id": (_i32, [_p]),
    "dkm_allreduce_init_rank": (_i32, [ctypes.c_char_p, _i32, _i32, _i32]),
    "dkm_allreduce_init": (_i32, [_i32, ctypes.POINTER(_i32)]),
    "dkm_allreduce_sum_f64": (_i32, [_p, _i64, _i32, _p]),
    "dkm_allreduce_finalize": (_i32, []),
    "dkm_allreduce_finalize_device": (_i32, [_i32]),
    "dkm_allreduce_available": (_i32, []),
    "dkm_allreduce_comm_info": (_i32, [_i32, ctypes.POINTER(_i32),
                                       ctypes.POINTER(_i32)]),
    "dkm_build_flags": (_i32, []),
    # host-side loaders (no GPU)
    "dkm_libsvm_count": (_i32, [_p, _i64, _i32, _p]),
    "dkm_libsvm_parse": (_i32, [_p, _i64, _i32, _p, _p, _p, _p, _p]),
    "dkm_txt_count": (_i32, [_p, _i64, _i32, _i32, _p]),
    "dkm_txt_parse": (_i32, [_p, _i64, _i32, _i64, _i32, _p, _p]),
}

_LIB = None


class DkmError(RuntimeError):
    pass


def load(path=None):
    """Load the shared library and bind every symbol (no GPU needed)."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise DkmError(
            "libdkm.so not found at %s: build it with "
            "`make -C dislib_amd/csrc` (or __graft_entry__.build())" % p)
    so = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(so, name)           # AttributeError if not exported
        fn.restype = res
        fn.argtypes = args
    if so.dkm_abi_version() != ABI_VERSION:
        raise DkmError("libdkm ABI %d != %d" % (so.dkm_abi_version(),
                                                 ABI_VERSION))
    if path is None:
        _LIB = so
    return so


def lib():
    """The library for compute calls: requires a visible ROCm GPU."""
    import torch
    if not torch.cuda.is_available():
        raise DkmError("dislib_amd needs an MI355X (ROCm) GPU: "
                       "torch.cuda.is_available() is False")
    return load()


def check(rc, what=""):
    if rc != 0:
        msg = _LIB.dkm_last_error().decode() if _LIB is not None else ""
        raise DkmError("%s failed (code %d): %s" % (what, rc, msg))
