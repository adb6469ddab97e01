"""ctypes binding of libignmp.so (include/ignmp.h).

The library is built in-tree by ``__graft_entry__.build()`` / ``python -m ignnition_amd.build``.
There is no fallback: if the shared object is missing or fails to load, importing this
module raises, and every compute call goes through the HIP kernels or fails loudly.
"""

from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# IGN_LIB_PATH selects an alternative in-tree build (used for A/B of compile flags)
LIB_PATH = os.environ.get("IGN_LIB_PATH", os.path.join(HERE, "libignmp.so"))

i32, i64, f32 = C.c_int32, C.c_int64, C.c_float


class EntityDesc(C.Structure):
    _fields_ = [("hidden_dim", i32), ("feature_total", i32)]


class DenseDesc(C.Structure):
    _fields_ = [("units", i32), ("activation", i32), ("use_bias", i32), ("l2", f32)]


class SourceDesc(C.Structure):
    _fields_ = [("entity", i32), ("adjacency", i32), ("interleave", i32), ("msg_num_inputs", i32),
                ("msg_inputs", C.POINTER(i32)), ("msg_param_dim", i32), ("msg_num_layers", i32),
                ("msg_layers", C.POINTER(DenseDesc))]


class MPDesc(C.Structure):
    _fields_ = [("dst_entity", i32), ("aggregation", i32), ("concat_axis", i32), ("cell", i32),
                ("num_sources", i32), ("sources", C.POINTER(SourceDesc)), ("activation", i32)]


class CellDesc(C.Structure):
    _fields_ = [("input_dim", i32), ("units", i32)]


class ReadoutOpDesc(C.Structure):
    _fields_ = [("type", i32), ("num_inputs", i32), ("inputs", C.POINTER(i32)), ("mode", i32),
                ("adjacency", i32), ("num_dense", i32), ("dense", C.POINTER(DenseDesc))]


class PlanDesc(C.Structure):
    _fields_ = [("num_iterations", i32), ("num_entities", i32), ("entities", C.POINTER(EntityDesc)),
                ("num_adjacencies", i32), ("num_interleave", i32), ("num_mps", i32),
                ("mps", C.POINTER(MPDesc)), ("num_cells", i32), ("cells", C.POINTER(CellDesc)),
                ("num_readout_inputs", i32), ("readout_inputs", C.POINTER(i32)),
                ("num_dense", i32), ("dense", C.POINTER(DenseDesc)),
                ("num_readout_ops", i32), ("readout_ops", C.POINTER(ReadoutOpDesc))]


class BatchDesc(C.Structure):
    _fields_ = [("num_graphs", i32), ("num_nodes", C.POINTER(i64)), ("features", C.POINTER(C.POINTER(f32))),
                ("adj_edges", C.POINTER(i64)), ("adj_src", C.POINTER(C.POINTER(i64))),
                ("adj_dst", C.POINTER(C.POINTER(i64))), ("adj_seq", C.POINTER(C.POINTER(i64))),
                ("interleave_len", C.POINTER(i64)), ("interleave_idx", C.POINTER(C.POINTER(i64))),
                ("halo_rows", C.POINTER(i64)), ("adj_params", C.POINTER(C.POINTER(f32))),
                ("index_bytes", i32)]   # ABI 13: 0/8 int64 index arrays, 4 int32


class DatasetDesc(C.Structure):
    _fields_ = [("num_features", i32), ("features", C.POINTER(C.c_char_p)), ("output_name", C.c_char_p),
                ("num_adjacencies", i32), ("adj_name", C.POINTER(C.c_char_p)), ("adj_src", C.POINTER(C.c_char_p)),
                ("adj_dst", C.POINTER(C.c_char_p)), ("adj_params", C.POINTER(i32)),
                ("num_interleave", i32), ("il_name", C.POINTER(C.c_char_p)), ("il_dst", C.POINTER(C.c_char_p)),
                ("num_additional", i32), ("additional", C.POINTER(C.c_char_p))]


class BatchInfo(C.Structure):
    _fields_ = [("num_graphs", i64), ("predictions", i64), ("output_units", i64), ("edges_per_forward", i64),
                ("gru_steps_per_forward", i64), ("rows", i64 * 8)]


class ResidentInfo(C.Structure):
    _fields_ = [("active", i32), ("form", i32), ("lds_bytes", i64), ("tile_steps", i64), ("union_tiles", i64),
                ("seg_rows", i64), ("messages", i64), ("bytes_compulsory", C.c_double),
                ("bytes_roundtrip", C.c_double), ("bytes_stage", C.c_double), ("flops", C.c_double),
                ("mfma_bf16", C.c_double), ("mfma_f32", C.c_double), ("workgroups", i32),
                ("graphs_per_workgroup", i32)]


class Stats(C.Structure):
    _fields_ = [("kinds", i32), ("launches", i64 * 8), ("ms", C.c_double * 8), ("flops", C.c_double * 8),
                ("bytes", C.c_double * 8), ("mfma_bf16", C.c_double * 8), ("mfma_f32", C.c_double * 8)]


KERNEL_KINDS = ["init_state", "seq_gru", "sum_gru", "readout", "project", "other", "mp_resident"]

MSG_INPUT = {"hs_source": 0, "hs_dest": 1, "edge_params": 2}
AGGR = {"sum": 0, "ordered": 1, "interleave": 2, "concat": 3, "attention": 4, "convolution": 5}
READOUT_OP = {"neural_network": 0, "pooling": 1, "product": 2, "extend_adjacencies": 3}
POOLING = {"sum": 0, "mean": 1, "max": 2}
PRODUCT = {"element_wise": 0, "dot_product": 1}
ACT = {None: 0, "None": 0, "linear": 0, "relu": 1, "selu": 2, "sigmoid": 3, "tanh": 4}

# every symbol declared in include/ignmp.h
SYMBOLS = ["ign_abi_version", "ign_last_error", "ign_device_count", "ign_plan_create", "ign_plan_destroy",
           "ign_plan_num_params", "ign_plan_num_param_tensors", "ign_plan_param_tensor", "ign_plan_set_params",
           "ign_plan_set_timing", "ign_plan_set_stream", "ign_plan_trim_cache", "ign_batch_create", "ign_batch_destroy", "ign_batch_info",
           "ign_forward", "ign_synchronize", "ign_batch_predictions", "ign_batch_state", "ign_stats",
           "ign_forward_begin", "ign_forward_mp", "ign_forward_end", "ign_batch_mp_split", "ign_batch_bind_state",
           "ign_batch_state_slot", "ign_gather_rows", "ign_plan_set_timing_kinds",
           "ign_batch_enable_training", "ign_forward_train", "ign_backward", "ign_mse_loss", "ign_l2_loss",
           "ign_adam_step", "ign_plan_get_params", "ign_dataset_open", "ign_dataset_close", "ign_dataset_size",
           "ign_dataset_error", "ign_dataset_gather", "ign_dataset_get", "ign_dataset_batch_create",
           "ign_dataset_batch_get", "ign_dataset_batch_get_narrow", "ign_dataset_batch_destroy", "ign_plan_create_json", "ign_plan_describe_json", "ign_forward_train_begin", "ign_forward_train_mp",
           "ign_forward_train_end", "ign_backward_begin", "ign_backward_mp", "ign_backward_end",
           "ign_batch_train_buffers", "ign_batch_read_predictions", "ign_batch_resident_info"]

ABI_VERSION = 13
PART = {"all": 0, "interior": 1, "boundary": 2}


def _load():
    # torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's): whichever loads first
    # serves the whole process.  Load torch's first so that the engine and torch share one HIP
    # runtime (streams and device pointers cross between them in partition.py); with /opt/rocm's
    # loaded first, torch finds no devices.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError("libignmp.so not built: run `python -m ignnition_amd.build` (or __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    P, VP = C.POINTER, C.c_void_p
    sig = {
        "ign_abi_version": (C.c_int, []),
        "ign_last_error": (C.c_char_p, []),
        "ign_device_count": (C.c_int, [P(i32)]),
        "ign_plan_create": (C.c_int, [P(PlanDesc), i32, P(VP)]),
        "ign_plan_destroy": (None, [VP]),
        "ign_plan_num_params": (C.c_int, [VP, P(i64)]),
        "ign_plan_num_param_tensors": (C.c_int, [VP, P(i32)]),
        "ign_plan_param_tensor": (C.c_int, [VP, i32, P(i32), P(i32), P(i64), P(i32), P(i32)]),
        "ign_plan_set_params": (C.c_int, [VP, VP, i32]),
        "ign_plan_set_timing": (C.c_int, [VP, i32]),
        "ign_plan_set_stream": (C.c_int, [VP, VP]),
        "ign_plan_trim_cache": (C.c_int, [VP]),
        "ign_batch_create": (C.c_int, [VP, P(BatchDesc), P(VP)]),
        "ign_batch_destroy": (None, [VP]),
        "ign_batch_info": (C.c_int, [VP, P(BatchInfo)]),
        "ign_forward": (C.c_int, [VP, VP, VP]),
        "ign_synchronize": (C.c_int, [VP]),
        "ign_batch_predictions": (C.c_int, [VP, P(VP)]),
        "ign_batch_state": (C.c_int, [VP, VP, i32, VP]),
        "ign_stats": (C.c_int, [VP, P(Stats)]),
        "ign_forward_begin": (C.c_int, [VP, VP]),
        "ign_forward_mp": (C.c_int, [VP, VP, i32, i32]),
        "ign_forward_end": (C.c_int, [VP, VP, VP]),
        "ign_batch_mp_split": (C.c_int, [VP, i32, P(i64), P(i64)]),
        "ign_batch_bind_state": (C.c_int, [VP, VP, i32, VP, VP, i64]),
        "ign_batch_state_slot": (C.c_int, [VP, i32, P(i32)]),
        "ign_gather_rows": (C.c_int, [VP, VP, i64, VP, i64, i32, VP]),
        "ign_plan_set_timing_kinds": (C.c_int, [VP, C.c_uint32]),
        "ign_batch_enable_training": (C.c_int, [VP, VP]),
        "ign_forward_train": (C.c_int, [VP, VP, VP]),
        "ign_backward": (C.c_int, [VP, VP, VP, VP]),
        "ign_mse_loss": (C.c_int, [VP, VP, VP, i64, VP, P(C.c_double)]),
        "ign_l2_loss": (C.c_int, [VP, P(C.c_double)]),
        "ign_adam_step": (C.c_int, [VP, VP, VP, VP, i64, f32, f32, f32, f32]),
        "ign_plan_get_params": (C.c_int, [VP, VP]),
        "ign_dataset_open": (C.c_int, [C.c_char_p, P(DatasetDesc), i32, P(VP)]),
        "ign_dataset_close": (None, [VP]),
        "ign_dataset_size": (C.c_int, [VP, P(i64), P(i32)]),
        "ign_dataset_error": (C.c_char_p, [VP, i32]),
        "ign_dataset_gather": (C.c_int, [VP, P(i64), i32]),
        "ign_dataset_get": (C.c_int, [VP, C.c_char_p, P(i32), P(VP), P(i64), P(P(i64))]),
        "ign_dataset_batch_create": (C.c_int, [VP, P(i64), i32, P(VP)]),
        "ign_dataset_batch_get": (C.c_int, [VP, C.c_char_p, P(i32), P(VP), P(i64), P(P(i64))]),
        "ign_dataset_batch_get_narrow": (C.c_int, [VP, C.c_char_p, P(i32), P(VP), P(i64), P(P(i64))]),
        "ign_dataset_batch_destroy": (None, [VP]),
        "ign_plan_create_json": (C.c_int, [C.c_char_p, C.c_char_p, i32, P(VP)]),
        "ign_plan_describe_json": (C.c_int, [VP, C.c_char_p, i64, P(i64)]),
        "ign_forward_train_begin": (C.c_int, [VP, VP]),
        "ign_forward_train_mp": (C.c_int, [VP, VP]),
        "ign_forward_train_end": (C.c_int, [VP, VP, VP]),
        "ign_backward_begin": (C.c_int, [VP, VP, VP, VP, f32]),
        "ign_backward_mp": (C.c_int, [VP, VP]),
        "ign_backward_end": (C.c_int, [VP, VP]),
        "ign_batch_train_buffers": (C.c_int, [VP, i32, P(VP), P(VP)]),
        "ign_batch_read_predictions": (C.c_int, [VP, VP, VP]),
        "ign_batch_resident_info": (C.c_int, [VP, P(ResidentInfo)]),
    }
    # an A/B build of an older tree may lack newer entry points: only the A/B tools, which set
    # IGN_AB_LIB=1 next to IGN_LIB_PATH, skip them; any other library must export every symbol
    ab = os.environ.get("IGN_AB_LIB") == "1"
    for name, (res, args) in sig.items():
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()
if lib.ign_abi_version() != ABI_VERSION:
    if os.environ.get("IGN_AB_LIB") != "1":
        raise ImportError("libignmp.so ABI %d, bindings expect %d: rebuild (python -m ignnition_amd.build)"
                          % (lib.ign_abi_version(), ABI_VERSION))
    # A/B against an older build: the ctypes structs (BatchInfo, Stats, ResidentInfo) are this
    # ABI's layouts, so fields the older library does not fill read as garbage -- say so loudly
    import sys as _sys
    print("ignnition_amd: WARNING: IGN_AB_LIB=1 loads %s with ABI %d, the bindings are ABI %d; struct "
          "layouts may differ" % (os.environ.get("IGN_LIB_PATH", "libignmp.so"), lib.ign_abi_version(), ABI_VERSION),
          file=_sys.stderr)


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libignmp error %d: %s" % (code, msg))
        self.code = code


def check(rc):
    if rc != 0:
        raise EngineError(rc, lib.ign_last_error().decode(errors="replace"))
    return rc
