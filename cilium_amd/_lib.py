"""ctypes binding of libgpuflow (include/gpuflow.h).

The shared library is built in-tree by ``__graft_entry__.build()``
(``cilium_amd/libgpuflow.so``).  There is no fallback: if it is missing the
import fails loudly.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgpuflow.so")
# diagnostic / variant builds only (tools/diag.sh, tools/variants.sh); never set in tests, smoke or bench runs
if os.environ.get("GPUFLOW_DIAG_LIB"):
    LIB_PATH = os.environ["GPUFLOW_DIAG_LIB"]

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libgpuflow.so not found at {LIB_PATH}; run `python -c 'import __graft_entry__ as g; g.build()'`")

# One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64
# (SONAME libamdhip64.so.7).  Loading torch first lets that copy satisfy
# libgpuflow's libamdhip64.so.7 dependency; loading libgpuflow first would map
# /opt/rocm's runtime as a second, separate HIP/HSA runtime next to torch's.
try:
    import torch  # noqa: F401
except ImportError:   # hosts without torch (e.g. a cgo agent) use /opt/rocm's runtime
    pass

lib = C.CDLL(LIB_PATH)

GF_MAX_L4_INGRESS = 64
GF_STATS_WORDS = 512


class gf_map_info(C.Structure):
    _fields_ = [("map_type", C.c_uint32), ("key_size", C.c_uint32), ("value_size", C.c_uint32),
                ("max_entries", C.c_uint32), ("map_flags", C.c_uint32), ("n_entries", C.c_uint32),
                ("device_bytes", C.c_uint64), ("xfer_d2h", C.c_uint64), ("xfer_h2d", C.c_uint64)]


class gf_pkt_cols(C.Structure):
    _fields_ = [("n", C.c_uint32), ("len", C.c_void_p), ("ethertype", C.c_void_p),
                ("saddr4", C.c_void_p), ("daddr4", C.c_void_p), ("proto", C.c_void_p),
                ("l4_off", C.c_void_p), ("l4w0", C.c_void_p), ("l4w3", C.c_void_p),
                ("saddr6", C.c_void_p), ("daddr6", C.c_void_p), ("src_identity", C.c_void_p),
                ("ifindex", C.c_void_p), ("lxc_id", C.c_void_p), ("tc_index", C.c_void_p),
                ("flow_hash", C.c_void_p)]


class gf_frames(C.Structure):
    _fields_ = [("n", C.c_uint32), ("snap_stride", C.c_uint32), ("snap", C.c_void_p), ("len", C.c_void_p)]


class gf_pkt_cols_out(C.Structure):
    _fields_ = [("ethertype", C.c_void_p), ("saddr4", C.c_void_p), ("daddr4", C.c_void_p),
                ("proto", C.c_void_p), ("l4_off", C.c_void_p), ("l4w0", C.c_void_p), ("l4w3", C.c_void_p),
                ("saddr6", C.c_void_p), ("daddr6", C.c_void_p)]


class gf_xdp_cfg(C.Structure):
    _fields_ = [("cidr4_hmap", C.c_int), ("cidr4_lmap", C.c_int), ("cidr6_hmap", C.c_int),
                ("cidr6_lmap", C.c_int), ("lxc_map", C.c_int)]


class gf_lb_cfg(C.Structure):
    _fields_ = [("lb4_services", C.c_int), ("lb6_services", C.c_int), ("flags", C.c_uint32),
                ("redirect_ifindex", C.c_uint32)]


class gf_l4_allow(C.Structure):
    _fields_ = [("port", C.c_uint16), ("proxy", C.c_uint16), ("nexthdr", C.c_uint8), ("pad", C.c_uint8 * 3)]


class gf_lxc_cfg(C.Structure):
    _fields_ = [("lxc_id", C.c_uint32), ("seclabel", C.c_uint32), ("policy_map", C.c_int),
                ("ct_map4", C.c_int), ("ct_map6", C.c_int), ("cidr4_ingress_map", C.c_int),
                ("cidr6_ingress_map", C.c_int), ("revnat4_map", C.c_int), ("revnat6_map", C.c_int),
                ("flags", C.c_uint32), ("n_l4_ingress", C.c_uint32),
                ("l4_ingress", gf_l4_allow * GF_MAX_L4_INGRESS), ("lxc_mac", C.c_uint8 * 6),
                ("node_mac", C.c_uint8 * 6), ("lxc_ipv4", C.c_uint32), ("lb4_services", C.c_int),
                ("ipcache_map", C.c_int), ("cidr4_egress_map", C.c_int), ("n_portmap", C.c_uint32),
                ("portmap", C.c_uint16 * 32), ("n_l4_egress", C.c_uint32),
                ("l4_egress", gf_l4_allow * GF_MAX_L4_INGRESS), ("lxc_ip6", C.c_uint8 * 16),
                ("lb6_services", C.c_int), ("cidr6_egress_map", C.c_int)]


class gf_prof_rec(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("count", C.c_uint32), ("pad", C.c_uint32), ("total_ms", C.c_double)]


class gf_node_cfg(C.Structure):
    _fields_ = [("host_ifindex", C.c_uint32), ("proxy4_map", C.c_int), ("proxy6_map", C.c_int),
                ("ipv4_gateway", C.c_uint32), ("host_ip6", C.c_uint8 * 16), ("host_mac", C.c_uint8 * 6),
                ("node_mac", C.c_uint8 * 6), ("lxc_map", C.c_int), ("ipv4_cluster_range", C.c_uint32),
                ("ipv4_cluster_mask", C.c_uint32), ("ipv4_loopback", C.c_uint32), ("ipv4_mask", C.c_uint32),
                ("encap_ifindex", C.c_uint32), ("tunnel_map", C.c_int), ("router_ip6", C.c_uint8 * 16)]


class gf_netdev_cfg(C.Structure):
    _fields_ = [("lxc_map", C.c_int), ("flags", C.c_uint32), ("fixed_secctx", C.c_uint32),
                ("router_ip6", C.c_uint8 * 16), ("ingress_ifindex", C.c_uint32)]


class gf_pipeline_cfg(C.Structure):
    _fields_ = [("xdp_prog", C.c_int), ("lb_prog", C.c_int), ("netdev", gf_netdev_cfg), ("policy_array", C.c_int)]


class gf_pipe_batch(C.Structure):
    _fields_ = [("frames", gf_frames), ("tc_index", C.c_void_p), ("flow_hash", C.c_void_p)]


class gf_lxc_batch(C.Structure):
    _fields_ = [("frames", gf_frames), ("lxc_id", C.c_void_p), ("flow_hash", C.c_void_p)]


class gf_event_ring(C.Structure):
    _fields_ = [("records", C.c_void_p), ("capacity", C.c_uint32), ("count", C.c_void_p)]


GF_EVENT_RECORD = 160


def _sig(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


VP = C.c_void_p
_sig("gf_map_create", C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32)
_sig("gf_map_update_elem", C.c_int, C.c_int, VP, VP, C.c_uint64)
_sig("gf_map_lookup_elem", C.c_int, C.c_int, VP, VP)
_sig("gf_map_delete_elem", C.c_int, C.c_int, VP)
_sig("gf_map_get_next_key", C.c_int, C.c_int, VP, VP)
_sig("gf_map_update_batch", C.c_int, C.c_int, VP, VP, C.c_uint32, C.c_uint64, C.POINTER(C.c_uint32))
_sig("gf_map_get_info", C.c_int, C.c_int, C.POINTER(gf_map_info))
_sig("gf_map_lookup_batch", C.c_int, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), VP, VP,
     C.POINTER(C.c_uint32))
_sig("gf_obj_pin", C.c_int, C.c_int, C.c_char_p)
_sig("gf_obj_get", C.c_int, C.c_char_p)
_sig("gf_obj_close", C.c_int, C.c_int)
_sig("gf_obj_unpin", C.c_int, C.c_char_p)
_sig("gf_now_sec", C.c_uint32)
_sig("gf_parse_frames", C.c_int, C.POINTER(gf_frames), C.POINTER(gf_pkt_cols_out), VP)
_sig("gf_xdp_prog_load", C.c_int, C.POINTER(gf_xdp_cfg))
_sig("gf_xdp_classify", C.c_int, C.c_int, C.POINTER(gf_pkt_cols), VP, VP)
_sig("gf_lb_prog_load", C.c_int, C.POINTER(gf_lb_cfg))
_sig("gf_lb_classify", C.c_int, C.c_int, C.POINTER(gf_pkt_cols), VP, VP, VP)
_sig("gf_lxc_prog_load", C.c_int, C.POINTER(gf_lxc_cfg))
_sig("gf_policy_array_create", C.c_int)
_sig("gf_policy_array_update", C.c_int, C.c_int, C.c_uint32, C.c_int)
_sig("gf_node_config", C.c_int, C.POINTER(gf_node_cfg))
_sig("gf_policy_ingress_classify", C.c_int, C.c_int, C.POINTER(gf_pkt_cols), C.c_uint32, VP, VP)
_sig("gf_policy_ingress_classify_batches", C.c_int, C.c_int, C.c_uint32, C.POINTER(C.POINTER(gf_pkt_cols)),
     C.POINTER(C.c_uint32), C.POINTER(VP), VP)
_sig("gf_pipeline_load", C.c_int, C.POINTER(gf_pipeline_cfg))
_sig("gf_pipeline_classify", C.c_int, C.c_int, C.POINTER(gf_pipe_batch), C.c_uint32, VP, VP, VP, VP)
_sig("gf_ct_gc", C.c_int, C.c_int, C.c_uint32, VP)


class gf_ct_evict_rec(C.Structure):
    _fields_ = [("seq", C.c_uint32), ("now_sec", C.c_uint32), ("age_cut", C.c_uint32), ("pad", C.c_uint32),
                ("hand_line", C.c_uint64), ("lines", C.c_uint64), ("evicted", C.c_uint64)]


_sig("gf_ct_evict_log", C.c_int, C.c_int, C.POINTER(gf_ct_evict_rec), C.c_uint32)
_sig("gf_pipeline_partition", C.c_int, C.c_int, C.POINTER(gf_pipe_batch), C.c_uint32, C.c_uint32, VP, VP, VP, VP)
_sig("gf_lxc_egress_classify", C.c_int, C.c_int, C.POINTER(gf_lxc_batch), C.c_uint32, VP, VP, VP)
_sig("gf_set_event_ring", C.c_int, C.POINTER(gf_event_ring))
_sig("gf_set_stats_sink", C.c_int, VP)
_sig("gf_prof_enable", C.c_int, C.c_int)
_sig("gf_prof_read", C.c_int, C.POINTER(gf_prof_rec), C.c_int)
_sig("gf_dev_alloc", VP, C.c_size_t)
_sig("gf_dev_free", C.c_int, VP)
_sig("gf_memcpy_h2d", C.c_int, VP, VP, C.c_size_t, VP)
_sig("gf_memcpy_d2h", C.c_int, VP, VP, C.c_size_t, VP)
_sig("gf_stream_sync", C.c_int, VP)
_sig("gf_device_count", C.c_int)
_sig("gf_version", C.c_char_p)
_sig("gf_build_id", C.c_char_p)

# Every symbol the C header declares (checked by tests/test_abi.py).
EXPORTED = [
    "gf_map_create", "gf_map_update_elem", "gf_map_lookup_elem", "gf_map_delete_elem",
    "gf_map_get_next_key", "gf_map_update_batch", "gf_map_lookup_batch", "gf_map_get_info", "gf_obj_pin", "gf_obj_get",
    "gf_obj_close", "gf_obj_unpin", "gf_now_sec", "gf_parse_frames", "gf_xdp_prog_load",
    "gf_xdp_classify", "gf_lb_prog_load", "gf_lb_classify", "gf_lxc_prog_load",
    "gf_policy_array_create", "gf_policy_array_update", "gf_node_config",
    "gf_policy_ingress_classify", "gf_policy_ingress_classify_batches", "gf_pipeline_load", "gf_pipeline_classify", "gf_pipeline_partition", "gf_lxc_egress_classify", "gf_ct_gc", "gf_ct_evict_log", "gf_set_event_ring", "gf_set_stats_sink", "gf_prof_enable", "gf_prof_read", "gf_dev_alloc", "gf_dev_free",
    "gf_memcpy_h2d", "gf_memcpy_d2h", "gf_stream_sync", "gf_device_count", "gf_version", "gf_build_id",
]

BUILD_ID = lib.gf_build_id().decode()


def source_sha():
    """sha256 prefix of the library's sources as they are in the tree now (the
    same digest __graft_entry__.build() compiles in as gf_build_id())."""
    import hashlib
    root = os.path.dirname(_HERE)
    files = [os.path.join(_HERE, "csrc", f) for f in sorted(os.listdir(os.path.join(_HERE, "csrc")))
             if f.endswith((".hip", ".cpp", ".h"))] + [os.path.join(root, "include", "gpuflow.h")]
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


# The library must be the one the tree's sources build: a stale binary fails here
# instead of running.  Variant builds of tools/ (GPUFLOW_DIAG_LIB) carry the same
# digest plus "+<variant>" (tools/variants.sh, tools/diag.sh), so a variant compiled
# from older sources — whose structs may no longer match this binding — fails too.
if os.path.isdir(os.path.join(_HERE, "csrc")):
    _want = source_sha()
    if os.environ.get("GPUFLOW_DIAG_LIB"):
        if not BUILD_ID.startswith(_want + "+"):
            raise ImportError(f"variant library {LIB_PATH} was built from sources {BUILD_ID}, the tree holds "
                              f"{_want}: rebuild it with tools/variant.sh")
    elif BUILD_ID != _want:
        raise ImportError(f"libgpuflow.so was built from sources {BUILD_ID}, the tree holds {_want}: "
                          "run `python -c 'import __graft_entry__ as g; g.build()'`")
