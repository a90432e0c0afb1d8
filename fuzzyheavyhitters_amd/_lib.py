"""ctypes binding of libfhh.so (C ABI in include/fhh.h).

The product path is the HIP library only: if libfhh.so is missing or fails to load, every
entry point raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import sys
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfhh.so")
# same-box A/B of two builds (tools/ab_builds.sh): load another copy of the library instead
if os.environ.get("FHH_LIB_PATH"):
    LIB_PATH = os.environ["FHH_LIB_PATH"]
_CSRC = os.path.join(_HERE, "csrc")
_LIB = None

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p

ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, u64p, ctypes.c_uint64, ctypes.c_void_p)

FHH_MAX_DIMS = 4

# value formats of fhh_node_sums_*_device (include/fhh.h)
FHH_VALS_FE_U64, FHH_VALS_FE_BLOCK, FHH_VALS_FE255_LIMBS, FHH_VALS_FE255_BLOCKPAIR = 0, 1, 2, 3
# reductions of a multi-device collection (fhh_shard_info)
FHH_REDUCE_NAMES = {0: "none", 1: "host", 2: "rccl"}

# every symbol include/fhh.h declares
EXPORTS = [
    "fhh_create", "fhh_destroy", "fhh_last_error", "fhh_reset", "fhh_set_client_base",
    "fhh_add_keys", "fhh_add_keys_bincode", "fhh_gen_keys_pair", "fhh_num_clients", "fhh_export_keys",
    "fhh_tree_init", "fhh_tree_crawl", "fhh_tree_crawl_last", "fhh_node_sums_fe",
    "fhh_node_sums_fe255", "fhh_tree_prune", "fhh_tree_prune_last", "fhh_frontier_size",
    "fhh_final_shares", "fhh_export_states", "fhh_keep_values", "fhh_keep_values_last",
    "fhh_final_values", "fhh_sim_eq_count", "fhh_sim_ot_sums", "fhh_sim_crawl",
    "fhh_get_stats", "fhh_reset_stats", "fhh_set_timing", "fhh_device_info", "fhh_microbench", "fhh_microbench_gather", "fhh_microbench_hybrid", "fhh_sketch_set_impl", "fhh_sketch_plan",
    "fhh_debug_launch_gaps", "fhh_wave_profile_arm", "fhh_wave_profile_launches",
    "fhh_set_variant", "fhh_variant_info",
    "fhh_rccl_load", "fhh_comm_unique_id", "fhh_comm_create", "fhh_comm_destroy", "fhh_comm_allreduce_u64",
    "fhh_comm_info", "fhh_comm_create_hosted", "fhh_comm_last_error",
    "fhh_sketch_at_fe", "fhh_mul_cor_share_fe", "fhh_mul_cor_fe", "fhh_mul_out_share_fe", "fhh_mul_verify_fe",
    "fhh_sim_sketch_verify_fe", "fhh_sketch_at_fe255", "fhh_mul_cor_share_fe255", "fhh_mul_cor_fe255",
    "fhh_mul_out_share_fe255", "fhh_mul_verify_fe255", "fhh_sim_sketch_verify_fe255", "fhh_deal_triples_fe",
    "fhh_co15_sender_start", "fhh_co15_receiver", "fhh_co15_sender_finish", "fhh_base_ot_co15",
    "fhh_base_ot_last_error",
    "fhh_gc_equality_device", "fhh_gc_equality_host", "fhh_ot_extend_device", "fhh_ot_extend_host",
    "fhh_create_multi", "fhh_shard_info", "fhh_shard_ctx", "fhh_node_sums_fe_device", "fhh_node_sums_fe255_device",
    "fhh_gb_garble", "fhh_gb_ot_labels", "fhh_gb_ot_shares", "fhh_ev_ot_labels", "fhh_ev_evaluate", "fhh_ev_ot_shares",
    "fhh_party_node_sums", "fhh_party_bytes_sent", "fhh_gc_party_test_cfgs", "fhh_memcpy_device",
    "fhh_cot_extend_host", "fhh_cot_extend_ss_host", "fhh_gc_cot_host", "fhh_gt_cot_host", "fhh_gt_cot_ring32_host",
    "fhh_shard_plan",
]


class FhhStats(ctypes.Structure):
    _fields_ = [
        ("aes_blocks", ctypes.c_uint64),
        ("ref_evals", ctypes.c_uint64),
        ("expand_launches", ctypes.c_uint64),
        ("expand_ms", ctypes.c_double),
        ("expand_blocks_timed", ctypes.c_uint64),
        ("levels", ctypes.c_uint64),
        ("keygen_ms", ctypes.c_double),
        ("expand_launches_timed", ctypes.c_uint64),
        ("base_ot_ms", ctypes.c_double),
        ("allreduce_ms", ctypes.c_double),
        ("allreduce_timed", ctypes.c_uint64),
        ("gcot_ms", ctypes.c_double),
        ("gcot_timed", ctypes.c_uint64),
        ("base_ot_stall_ms", ctypes.c_double),
        ("base_ot_instances", ctypes.c_uint64),
    ]


class FhhSimConfig(ctypes.Structure):
    _fields_ = [
        ("threshold", ctypes.c_double),
        ("nclients_total", ctypes.c_uint64),
        ("mode", ctypes.c_uint32),
        ("levels", ctypes.c_uint32),
        ("prf_seed", ctypes.c_uint64),
        ("allreduce", ALLREDUCE_FN),
        ("allreduce_user", ctypes.c_void_p),
        ("xchg_dev", u64p),
        ("xchg_capacity", ctypes.c_uint64),
        ("level_children", u64p),
        ("level_kept", u64p),
        ("counts", u64p),
        ("counts_capacity", ctypes.c_uint64),
        ("host_loop", ctypes.c_uint32),
        ("init_capacity", ctypes.c_uint32),
        ("comm", ctypes.c_void_p),
        ("gc", ctypes.c_uint32),
        ("probe_n_levels", ctypes.c_uint32),
        ("probe_n_clients", ctypes.c_uint32),
        ("probe_levels", u32p),
        ("probe_clients", u64p),
        ("probe_capacity", ctypes.c_uint64),
        ("probe_seeds", u8p),
        ("probe_ty", u8p),
        ("probe_children", u64p),
        ("base_ot", ctypes.c_uint32),
        ("ot_ss_k", ctypes.c_uint32),
        ("table_ring32", ctypes.c_uint32),
    ]


SOURCES = ("fhh_kernels.hip", "fhh_sketch.hip", "fhh_gc.hip", "fhh_ot.hip", "fhh_loop.hip",
           "fhh_microbench.hip", "fhh_host.cpp", "fhh_gcot.cpp", "fhh_group.cpp", "fhh_comm.cpp", "fhh_base_ot.cpp")


class FhhSketchBatch(ctypes.Structure):
    _fields_ = [
        ("n_keys", ctypes.c_uint64),
        ("n_nodes", ctypes.c_uint32),
        ("force_sequential", ctypes.c_uint32),
        ("seeds_dev", ctypes.c_void_p),
        ("x_dev", ctypes.c_void_p * 2),
        ("kx_dev", ctypes.c_void_p * 2),
        ("mac_dev", ctypes.c_void_p * 2),
        ("mac2_dev", ctypes.c_void_p * 2),
        ("triples_dev", ctypes.c_void_p * 2),
        ("sketch_dev", ctypes.c_void_p * 2),
        ("ok_dev", ctypes.c_void_p),
        ("out_shares_dev", ctypes.c_void_p),
        ("level", ctypes.c_uint32),
        ("n_levels", ctypes.c_uint32),
        ("triples_levels", ctypes.c_uint32),
        ("pad_", ctypes.c_uint32),
        ("x_level_stride", ctypes.c_uint64),
    ]


class FhhSketchBatch255(ctypes.Structure):
    _fields_ = [
        ("n_keys", ctypes.c_uint64),
        ("n_nodes", ctypes.c_uint32),
        ("force_sequential", ctypes.c_uint32),
        ("seeds_dev", ctypes.c_void_p),
        ("x_dev", ctypes.c_void_p * 2),
        ("kx_dev", ctypes.c_void_p * 2),
        ("mac_dev", ctypes.c_void_p * 2),
        ("mac2_dev", ctypes.c_void_p * 2),
        ("triples_dev", ctypes.c_void_p * 2),
        ("sketch_dev", ctypes.c_void_p * 2),
        ("ok_dev", ctypes.c_void_p),
        ("out_shares_dev", ctypes.c_void_p),
        ("level", ctypes.c_uint32),
        ("pad_", ctypes.c_uint32),
    ]


class FhhGcBatch(ctypes.Structure):
    _fields_ = [
        ("groups", ctypes.c_uint64),
        ("clients", ctypes.c_uint32),
        ("words", ctypes.c_uint32),
        ("bits", ctypes.c_uint32),
        ("mask", ctypes.c_uint32),
        ("label_key", ctypes.c_uint8 * 16),
        ("delta", ctypes.c_uint8 * 16),
        ("label_nonce", ctypes.c_uint64),
        ("gate_base", ctypes.c_uint64),
        ("gb_planes_dev", ctypes.c_void_p),
        ("ev_planes_dev", ctypes.c_void_p),
        ("tables_dev", ctypes.c_void_p),
        ("gb_labels_dev", ctypes.c_void_p),
        ("ev_labels_dev", ctypes.c_void_p),
        ("decode_dev", ctypes.c_void_p),
        ("out_dev", ctypes.c_void_p),
    ]


class FhhOtBatch(ctypes.Structure):
    _fields_ = [
        ("m", ctypes.c_uint64),
        ("choices_dev", ctypes.c_void_p),
        ("x0_dev", ctypes.c_void_p),
        ("x1_dev", ctypes.c_void_p),
        ("delta", ctypes.c_uint8 * 16),
        ("out_dev", ctypes.c_void_p),
        ("base_seeds", ctypes.c_uint8 * (128 * 2 * 16)),
        ("base_choice", ctypes.c_uint8 * 16),
        ("tweak_base", ctypes.c_uint64),
    ]


class FhhGbCfg(ctypes.Structure):
    """fhh_gb_cfg: the garbler's (server 0's) own material for one chunk (include/fhh.h)."""
    _fields_ = [
        ("mask", ctypes.c_uint32),
        ("form", ctypes.c_uint32),   # FE levels: 0 garbled table (2d <= 4), 1 half-gates circuit
        ("base_chosen", ctypes.c_uint8 * (2 * 128 * 16)),
        ("base_choice", ctypes.c_uint8 * (2 * 16)),
        ("child_begin", ctypes.c_uint64),
        ("child_count", ctypes.c_uint64),
        ("ot_ss_k", ctypes.c_uint32),   # r06: 0 / 1 IKNP, 2 / 4 SoftSpoken (as the evaluator's)
        ("pad_", ctypes.c_uint32),
    ]


class FhhEvCfg(ctypes.Structure):
    """fhh_ev_cfg: the evaluator's (server 1's) own material: its base-OT key pairs, nothing else."""
    _fields_ = [
        ("base_pairs", ctypes.c_uint8 * (2 * 128 * 2 * 16)),
        ("form", ctypes.c_uint32),   # as FhhGbCfg.form (public)
        ("ot_ss_k", ctypes.c_uint32),   # r06: 0 / 1 IKNP, 2 / 4 SoftSpoken
        ("child_begin", ctypes.c_uint64),
        ("child_count", ctypes.c_uint64),
    ]


# fhh_cot_extend_host modes (include/fhh.h)
FHH_COT_LABELS, FHH_COT_FE, FHH_COT_FE255, FHH_COT_RAW = 1, 2, 3, 4


def build(verbose: bool = False) -> str:
    """Compile libfhh.so for gfx950 with hipcc (in-tree, travels to the GPU box): one object per
    source, compiled in parallel, then one link."""
    from concurrent.futures import ThreadPoolExecutor
    objdir = os.path.join(_HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall"]
    # kernel tuning defines are honoured only in an explicit A/B build (tools/ab_builds.sh sets both),
    # and announced, so a stray environment variable cannot change the product kernels silently
    extra = os.environ.get("FHH_EXTRA_DEFINES", "").split()
    if extra and os.environ.get("FHH_AB_BUILD") == "1":
        flags += ["-D" + d for d in extra]
        print(f"fhh build: A/B defines {extra}", file=sys.stderr)
    elif extra:
        print("fhh build: FHH_EXTRA_DEFINES ignored (set FHH_AB_BUILD=1 for an A/B build)", file=sys.stderr)

    def compile_one(f):
        obj = os.path.join(objdir, f + ".o")
        r = subprocess.run(["hipcc", *flags, "-c", os.path.join(_CSRC, f), "-o", obj], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {f}:\n" + r.stdout + r.stderr)
        return obj, r.stdout + r.stderr

    with ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 4)) as ex:
        res = list(ex.map(compile_one, SOURCES))
    r = subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *[o for o, _ in res], "-ldl", "-lcrypto",
                        "-o", LIB_PATH], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc link failed:\n" + r.stdout + r.stderr)
    if verbose:
        for _, msg in res:
            if msg:
                print(msg)
    return LIB_PATH


class FhhError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise FhhError(f"{LIB_PATH} not built: run __graft_entry__.build() (the HIP extension is required; "
                       "there is no CPU fallback)")
    # One HIP runtime per process: when PyTorch is present, load it first so libfhh.so's
    # libamdhip64.so.7 dependency binds to the copy torch ships (torch cannot initialise the
    # GPU after a second runtime has claimed the soname; the other order is the one that works).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    i = ctypes.c_int
    u32 = ctypes.c_uint32
    u64 = ctypes.c_uint64
    P = ctypes.POINTER
    sig = {
        "fhh_create": (i, [P(vp), u32, u32, i]),
        "fhh_create_multi": (i, [P(vp), u32, u32, P(i), i]),
        "fhh_shard_info": (i, [vp, i, P(i), P(i), u64p, u64p, P(i)]),
        "fhh_shard_ctx": (i, [vp, i, P(vp)]),
        "fhh_node_sums_fe_device": (i, [vp, P(vp), u64, u32, u64p]),
        "fhh_node_sums_fe255_device": (i, [vp, P(vp), u64, u32, u32p, u32p]),
        "fhh_gb_garble": (i, [vp, P(vp), u64p]),
        "fhh_gb_ot_labels": (i, [vp, P(FhhGbCfg), vp, u64, P(vp), u64p]),
        "fhh_gb_ot_shares": (i, [vp, vp, u64, P(vp), u64p]),
        "fhh_ev_ot_labels": (i, [vp, P(FhhEvCfg), P(vp), u64p]),
        "fhh_ev_evaluate": (i, [vp, vp, u64, vp, u64, P(vp), u64p]),
        "fhh_ev_ot_shares": (i, [vp, vp, u64]),
        "fhh_party_node_sums": (i, [vp, vp, vp]),
        "fhh_party_bytes_sent": (i, [vp, u64p]),
        "fhh_gc_party_test_cfgs": (i, [u64, u32, P(FhhGbCfg), P(FhhEvCfg)]),
        "fhh_cot_extend_host": (i, [vp, u64, u32, u8p, u8p, u32, u8p, u8p, u64, u8p, u8p, u8p, u8p]),
        "fhh_cot_extend_ss_host": (i, [vp, u32, u64, u32, u8p, u8p, u32, u8p, u8p, u64, u8p, u8p, u8p, u8p, u8p]),
        "fhh_gc_cot_host": (i, [vp, u64, u32, u8p, u8p, u32, u64, u8p, u8p, u64, u8p, u8p, u8p, u8p, u8p, u64p, u64p,
                                u64p]),
        "fhh_gt_cot_host": (i, [vp, u64, u32, u8p, u8p, u32, u64, u8p, u8p, u64, u8p, u8p, u64p, u64p, u64p]),
        "fhh_gt_cot_ring32_host": (i, [vp, u64, u32, u8p, u8p, u32, u64, u8p, u8p, u64, u8p, u8p, u64p, u64p, u64p]),
        "fhh_memcpy_device": (i, [i, vp, vp, u64]),
        "fhh_shard_plan": (i, [u64, i, u64p, u64p]),
        "fhh_destroy": (None, [vp]),
        "fhh_last_error": (ctypes.c_char_p, [vp]),
        "fhh_reset": (i, [vp]),
        "fhh_set_client_base": (i, [vp, u64]),
        "fhh_add_keys": (i, [vp, u64, u8p, u8p, u8p, u8p]),
        "fhh_gen_keys_pair": (i, [vp, vp, u64, u8p, u8p, u8p]),
        "fhh_add_keys_bincode": (i, [vp, u8p, u64]),
        "fhh_num_clients": (i, [vp, u64p]),
        "fhh_export_keys": (i, [vp, u8p, u8p, u8p, u8p]),
        "fhh_tree_init": (i, [vp]),
        "fhh_tree_crawl": (i, [vp, u64p, u64p]),
        "fhh_tree_crawl_last": (i, [vp, u64p, u64p]),
        "fhh_node_sums_fe": (i, [vp, u64p, u64p]),
        "fhh_node_sums_fe255": (i, [vp, u32p, u32p, u32p]),
        "fhh_tree_prune": (i, [vp, u8p, u64]),
        "fhh_tree_prune_last": (i, [vp, u8p, u64]),
        "fhh_frontier_size": (i, [vp, u64p, u64p]),
        "fhh_final_shares": (i, [vp, u64p, u32p, u8p, u32p]),
        "fhh_export_states": (i, [vp, u64p, u8p, u8p, u8p]),
        "fhh_keep_values": (i, [u64, u64p, u64p, u64, u8p]),
        "fhh_keep_values_last": (i, [u32, u32p, u32p, u64, u8p]),
        "fhh_final_values": (i, [u32p, u32p, u64, u32p]),
        "fhh_sim_eq_count": (i, [vp, vp, u64p]),
        "fhh_sim_ot_sums": (i, [vp, vp, u64, vp, vp]),
        "fhh_sim_crawl": (i, [vp, vp, P(FhhSimConfig)]),
        "fhh_get_stats": (i, [vp, P(FhhStats)]),
        "fhh_reset_stats": (i, [vp]),
        "fhh_set_timing": (i, [vp, i]),
        "fhh_device_info": (i, [i, ctypes.c_char_p, ctypes.c_size_t, P(i)]),
        "fhh_microbench": (i, [i, i, P(ctypes.c_double)]),
        "fhh_microbench_gather": (i, [i, i, ctypes.c_uint32, P(ctypes.c_double)]),
        "fhh_microbench_hybrid": (i, [i, i, P(ctypes.c_double)]),
        "fhh_sketch_set_impl": (i, [i]),
        "fhh_sketch_plan": (i, [u64, u32, u64, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int),
                                ctypes.POINTER(ctypes.c_int)]),
        "fhh_debug_launch_gaps": (i, [i, i, i, P(ctypes.c_double)]),
        "fhh_wave_profile_arm": (i, [i, vp, ctypes.c_uint32]),
        "fhh_wave_profile_launches": (i, [i, P(ctypes.c_uint32)]),
        "fhh_set_variant": (i, [vp, i]),
        "fhh_variant_info": (i, [i, ctypes.c_char_p, ctypes.c_size_t, P(i), P(i)]),
        "fhh_rccl_load": (i, [ctypes.c_char_p]),
        "fhh_comm_unique_id": (i, [u8p]),
        "fhh_comm_create": (i, [P(vp), i, i, u8p, i]),
        "fhh_comm_destroy": (None, [vp]),
        "fhh_comm_allreduce_u64": (i, [vp, vp, vp, u64, vp]),
        "fhh_comm_last_error": (ctypes.c_char_p, []),
        "fhh_comm_info": (i, [vp, P(i), P(i)]),
        "fhh_comm_create_hosted": (i, [P(vp), i, i, i, ALLREDUCE_FN, vp]),
        "fhh_sketch_at_fe": (i, [vp, u64, u32, u8p, u64p, u64p, u64p]),
        "fhh_mul_cor_share_fe": (i, [vp, u64, u64p, u64p, u64p, u64p, u64p]),
        "fhh_mul_cor_fe": (i, [u64, u64p, u64p, u64p]),
        "fhh_mul_out_share_fe": (i, [vp, i, u64, u64p, u64p, u64p, u64p, u64p, u64p]),
        "fhh_mul_verify_fe": (i, [u64, u64p, u64p, u8p]),
        "fhh_sim_sketch_verify_fe": (i, [vp, P(FhhSketchBatch)]),
        "fhh_sketch_at_fe255": (i, [vp, u64, u32, u8p, u32p, u32p, u32p]),
        "fhh_mul_cor_share_fe255": (i, [vp, u64, u32p, u32p, u32p, u32p, u32p]),
        "fhh_mul_cor_fe255": (i, [u64, u32p, u32p, u32p]),
        "fhh_mul_out_share_fe255": (i, [vp, i, u64, u32p, u32p, u32p, u32p, u32p, u32p]),
        "fhh_mul_verify_fe255": (i, [u64, u32p, u32p, u8p]),
        "fhh_sim_sketch_verify_fe255": (i, [vp, P(FhhSketchBatch255)]),
        "fhh_deal_triples_fe": (i, [vp, u64, u32, u64, vp, vp]),
        "fhh_co15_sender_start": (i, [u8p, u8p]),
        "fhh_co15_receiver": (i, [u32, u8p, u8p, u8p, u8p, u8p]),
        "fhh_co15_sender_finish": (i, [u32, u8p, u8p, u8p]),
        "fhh_base_ot_co15": (i, [u32, u8p, u8p, u8p, u8p]),
        "fhh_base_ot_last_error": (ctypes.c_char_p, []),
        "fhh_gc_equality_device": (i, [vp, P(FhhGcBatch)]),
        "fhh_ot_extend_device": (i, [vp, P(FhhOtBatch)]),
        "fhh_ot_extend_host": (i, [vp, u64, u8p, u8p, u8p, u8p, u8p, u8p, u64, u8p, u8p, u8p, u8p]),
        "fhh_gc_equality_host": (i, [vp, u64, u32, u8p, u8p, u32, u8p, u8p, u64, u64, u8p, u8p, u8p, u8p, u8p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def check(rc: int, ctx=None):
    if rc != 0:
        msg = lib().fhh_last_error(ctx)
        raise FhhError(f"fhh error {rc}: {msg.decode() if msg else ''}")


def ptr(a, t=u8p):
    """Pointer to a C-contiguous numpy array (or None)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data_as(t)
