# SPDX-License-Identifier: Apache-2.0
"""ctypes mirror of include/dpgpu.h and the library loaders.

The product library is ``dataplane_amd/lib/libdpgpu.so`` (HIP kernels +
C ABI).  It is loaded from the source tree only; if it is missing or a GPU is
not present the calls fail loudly -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")

ABI_VERSION = 7
HEADROOM = 96

# DoneReason (net/src/packet/meta.rs:84-119)
DONE_NAMES = [
    "InternalFailure", "InterfaceUnknown", "InterfaceDetached", "InterfaceAdmDown",
    "InterfaceOperDown", "InterfaceUnsupported", "NotEthernet", "Unhandled", "MacNotForUs",
    "InvalidDstMac", "MissingEtherType", "NotIp", "RouteFailure", "RouteDrop",
    "HopLimitExceeded", "MissL2resolution", "VxlanDecapFailure", "VxlanEncapFailure",
    "Filtered", "AclDropped", "NatOutOfResources", "FlowCapacityExceeded",
    "NatUnsupportedProto", "NatFailure", "NatNotPortForwarded", "Malformed", "Unroutable",
    "InvalidChecksum", "IcmpErrorIncomplete", "InternalDrop", "Local", "Delivered",
    "DeparseError", "NoHeadRoom",
]
DONE = {n: i for i, n in enumerate(DONE_NAMES)}
DONE_COUNT = len(DONE_NAMES)
DONE_NONE = 255

# MetaFlags (net/src/packet/meta.rs:121-136)
META = dict(INITIALIZED=1 << 0, IS_L2_BCAST=1 << 1, NATTED_SRC=1 << 2, NATTED_DST=1 << 3,
            REFR_CHKSUM=1 << 4, KEEP=1 << 5, IS_OVERLAY=1 << 6, REQ_MASQUERADE=1 << 7,
            REQ_PORT_FORWARDING=1 << 8, REQ_STATIC_NAT_SRC=1 << 9, REQ_STATIC_NAT_DST=1 << 10)

IN_SEEDED_OVERLAY = 1

PKT_IN = np.dtype([("off", "<u4"), ("len", "<u2"), ("flags", "<u2"), ("iif", "<u4"),
                   ("src_vni", "<u4")])
# dp_pkt_out_t: what the driver needs to transmit or drop a packet (always written)
PKT_OUT = np.dtype([("off", "<u4"), ("len", "<u2"), ("done", "u1"), ("acl", "u1"),
                    ("oif", "<u4"), ("meta_flags", "<u2"), ("pad", "<u2")])
# dp_pkt_meta_t: the rest of PacketMeta (optional array)
PKT_META = np.dtype([("dst_vni", "<u4"), ("src_vni", "<u4"), ("fib_entry", "<u4"),
                     ("acl_rule", "<u4"), ("vrf", "<u4"), ("pm_flags", "u1"), ("dscp", "u1"),
                     ("ecn", "u1"), ("nh_family", "u1"), ("nh_addr", "u1", 16),
                     ("flow_ref", "<u8")])
assert PKT_IN.itemsize == 16 and PKT_OUT.itemsize == 16 and PKT_META.itemsize == 48
# one packet's whole result (test / host convenience): dp_pkt_out_t then dp_pkt_meta_t
PKT_RES = np.dtype(PKT_OUT.descr + PKT_META.descr)
assert PKT_RES.itemsize == 64
PM_HAS_VRF, PM_HAS_NH, PM_HAS_DSCP = 1, 2, 4


def join_results(out: np.ndarray, meta: np.ndarray) -> np.ndarray:
    """PKT_RES records from a dp_pkt_out_t array and a dp_pkt_meta_t array."""
    res = np.zeros(len(out), dtype=PKT_RES)
    for f in PKT_OUT.names:
        res[f] = out[f]
    for f in PKT_META.names:
        res[f] = meta[f]
    return res


def nh_text(r) -> str:
    """A PKT_RES / PKT_META record's next-hop address as text (nh_family 4 / 6)."""
    import ipaddress
    b = bytes(np.asarray(r["nh_addr"], dtype=np.uint8))
    return str(ipaddress.IPv4Address(b[:4]) if int(r["nh_family"]) == 4
               else ipaddress.IPv6Address(b))


def split_results(res: np.ndarray):
    """(dp_pkt_out_t array, dp_pkt_meta_t array) of PKT_RES records."""
    out = np.zeros(len(res), dtype=PKT_OUT)
    meta = np.zeros(len(res), dtype=PKT_META)
    for f in PKT_OUT.names:
        out[f] = res[f]
    for f in PKT_META.names:
        meta[f] = res[f]
    return out, meta

# Flow table (include/dpgpu.h "Flow table")
FLOW_TCP, FLOW_UDP, FLOW_ICMP_QUERY, FLOW_ICMP_OTHER = 1, 2, 3, 4
FLOW_ACTIVE, FLOW_CANCELLED, FLOW_EXPIRED, FLOW_DETACHED = 0, 1, 2, 3
FLOW_INITIATOR, FLOW_REQ_STATIC_NAT_SRC, FLOW_REQ_STATIC_NAT_DST = 1, 2, 4
FLOW_NONE = (1 << 64) - 1
FLOW_INSERTED, FLOW_REPLACED, EFLOWCAP = 0, 1, -28
ACL_SCOPE_FLOW, ACL_SCOPE_PACKET = 0, 1
FLOW_KEY = np.dtype([("src_vni", "<u4"), ("family", "u1"), ("kind", "u1"), ("pad", "<u2"),
                     ("sport", "<u2"), ("dport", "<u2"), ("src", "u1", 16), ("dst", "u1", 16)])
FLOW = np.dtype([("key", FLOW_KEY), ("dst_vni", "<u4"), ("flags", "<u4"), ("pad", "<u4"),
                 ("genid", "<i8"), ("expires_at", "<u8")], align=True)
FLOW_INFO = np.dtype([("ref", "<u8"), ("status", "<u4"), ("flags", "<u4"), ("dst_vni", "<u4"),
                      ("pad", "<u4"), ("genid", "<i8"), ("expires_at", "<u8"),
                      ("related", "<u8"), ("pf", "u1"), ("pf_status", "u1"), ("pf_port", "<u2"),
                      ("pf_rule", "<u4"), ("pf_family", "u1"), ("pad2", "u1", (7,)),
                      ("pf_ip", "u1", (16,)), ("masq", "u1"), ("masq_alloc", "u1"),
                      ("pad3", "<u2"), ("idle_timeout_s", "<u4")])
assert FLOW_KEY.itemsize == 44 and FLOW.itemsize == 72 and FLOW_INFO.itemsize == 88
# enum dp_pf_action / dp_nat_flow_status (include/dpgpu.h)
PF_NONE, PF_DST_NAT, PF_SRC_NAT = 0, 1, 2
(NFS_ONE_WAY, NFS_TWO_WAY, NFS_ESTABLISHED, NFS_RESET, NFS_C_CLOSING, NFS_S_CLOSING,
 NFS_C_HALF_CLOSE, NFS_S_HALF_CLOSE, NFS_LAST_ACK, NFS_CLOSED) = range(10)


class IpAddr(C.Structure):
    _fields_ = [("family", C.c_uint8), ("pad", C.c_uint8 * 3), ("addr", C.c_uint8 * 16)]


class Prefix(C.Structure):
    _fields_ = [("family", C.c_uint8), ("len", C.c_uint8), ("pad", C.c_uint8 * 2),
                ("addr", C.c_uint8 * 16)]


class Fib(C.Structure):
    _fields_ = [("vrf_id", C.c_uint32), ("flags", C.c_uint32), ("vtep_ip", IpAddr),
                ("vtep_mac", C.c_uint8 * 6), ("pad", C.c_uint8 * 2)]


class VniFib(C.Structure):
    _fields_ = [("vni", C.c_uint32), ("fib", C.c_uint32)]


class Instr(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("flags", C.c_uint32), ("ifindex", C.c_uint32),
                ("vni", C.c_uint32), ("addr", IpAddr), ("mac", C.c_uint8 * 6),
                ("pad", C.c_uint8 * 2)]


class FibEntry(C.Structure):
    _fields_ = [("first_instr", C.c_uint32), ("n_instr", C.c_uint32)]


class RouteNh(C.Structure):
    _fields_ = [("first_entry", C.c_uint32), ("n_entries", C.c_uint32)]


class Route(C.Structure):
    _fields_ = [("prefix", Prefix), ("fib", C.c_uint32), ("nh", C.c_uint32)]


class Iface(C.Structure):
    _fields_ = [("ifindex", C.c_uint32), ("admin_state", C.c_uint8), ("oper_state", C.c_uint8),
                ("iftype", C.c_uint8), ("attach", C.c_uint8), ("vrf_id", C.c_uint32),
                ("mac", C.c_uint8 * 6), ("pad", C.c_uint8 * 2)]


class Adjacency(C.Structure):
    _fields_ = [("addr", IpAddr), ("ifindex", C.c_uint32), ("mac", C.c_uint8 * 6),
                ("pad", C.c_uint8 * 2)]


class Rule(C.Structure):
    _fields_ = [("proto_val", C.c_uint8), ("proto_mask", C.c_uint8), ("family", C.c_uint8),
                ("gate", C.c_uint8), ("vni_a", C.c_uint32), ("vni_b", C.c_uint32),
                ("sport_lo", C.c_uint16), ("sport_hi", C.c_uint16), ("dport_lo", C.c_uint16),
                ("dport_hi", C.c_uint16), ("priority", C.c_uint32), ("src", Prefix),
                ("dst", Prefix), ("action", C.c_uint32), ("action2", C.c_uint32)]


class AclDefault(C.Structure):
    _fields_ = [("src_vni", C.c_uint32), ("dst_vni", C.c_uint32), ("action", C.c_uint32)]


class NatTable(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("src_vni", C.c_uint32), ("dst_vni", C.c_uint32),
                ("first_entry", C.c_uint32), ("n_entries", C.c_uint32)]


class NatEntry(C.Structure):
    _fields_ = [("prefix", Prefix), ("is_pat", C.c_uint32), ("first_port_range", C.c_uint32),
                ("n_port_ranges", C.c_uint32), ("first_range", C.c_uint32),
                ("n_ranges", C.c_uint32), ("pad", C.c_uint32), ("size", C.c_uint64)]


class PortRange(C.Structure):
    _fields_ = [("lo", C.c_uint16), ("hi", C.c_uint16)]


class NatRange(C.Structure):
    _fields_ = [("orig_lo_ip", C.c_uint8 * 4), ("orig_hi_ip", C.c_uint8 * 4),
                ("orig_lo_port", C.c_uint16), ("orig_hi_port", C.c_uint16),
                ("tgt_lo_ip", C.c_uint8 * 4), ("tgt_hi_ip", C.c_uint8 * 4),
                ("tgt_lo_port", C.c_uint16), ("tgt_hi_port", C.c_uint16),
                ("offset", C.c_uint64)]


def _arr(t):
    return [("%s" % t[0], C.POINTER(t[1])), ("n_%s" % t[0], t[2])]


class PortFwRule(C.Structure):
    _fields_ = [("src_vni", C.c_uint32), ("proto", C.c_uint8), ("pad", C.c_uint8 * 3),
                ("dst_vni", C.c_uint32), ("ext_lo", C.c_uint16), ("ext_hi", C.c_uint16),
                ("int_lo", C.c_uint16), ("int_hi", C.c_uint16), ("init_timeout_s", C.c_uint32),
                ("estab_timeout_s", C.c_uint32), ("ext_prefix", Prefix), ("int_prefix", Prefix)]


class MasqExpose(C.Structure):
    _fields_ = [("src_vni", C.c_uint32), ("dst_vni", C.c_uint32), ("idle_timeout_s", C.c_uint32),
                ("first_prefix", C.c_uint32), ("n_private", C.c_uint16), ("n_public", C.c_uint16),
                ("first_claim", C.c_uint32), ("n_claims", C.c_uint32)]


class MasqClaim(C.Structure):
    _fields_ = [("prefix", Prefix), ("lo", C.c_uint16), ("hi", C.c_uint16), ("protos", C.c_uint32)]


MASQ_TCP, MASQ_UDP = 1, 2
MASQ_REGION_ADDRS = 4096


class TablesDesc(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("pad0", C.c_uint32), ("genid", C.c_int64),
                ("fibs", C.POINTER(Fib)), ("n_fibs", C.c_uint32),
                ("vni_fibs", C.POINTER(VniFib)), ("n_vni_fibs", C.c_uint32),
                ("routes", C.POINTER(Route)), ("n_routes", C.c_uint64),
                ("route_nhs", C.POINTER(RouteNh)), ("n_route_nhs", C.c_uint32),
                ("entries", C.POINTER(FibEntry)), ("n_entries", C.c_uint32),
                ("instrs", C.POINTER(Instr)), ("n_instrs", C.c_uint32),
                ("ifaces", C.POINTER(Iface)), ("n_ifaces", C.c_uint32),
                ("adjs", C.POINTER(Adjacency)), ("n_adjs", C.c_uint32),
                ("acl_v4", C.POINTER(Rule)), ("n_acl_v4", C.c_uint32),
                ("acl_v6", C.POINTER(Rule)), ("n_acl_v6", C.c_uint32),
                ("acl_defaults", C.POINTER(AclDefault)), ("n_acl_defaults", C.c_uint32),
                ("ff_remote_v4", C.POINTER(Rule)), ("n_ff_remote_v4", C.c_uint32),
                ("ff_local_v4", C.POINTER(Rule)), ("n_ff_local_v4", C.c_uint32),
                ("ff_remote_v6", C.POINTER(Rule)), ("n_ff_remote_v6", C.c_uint32),
                ("ff_local_v6", C.POINTER(Rule)), ("n_ff_local_v6", C.c_uint32),
                ("nat_tables", C.POINTER(NatTable)), ("n_nat_tables", C.c_uint32),
                ("nat_entries", C.POINTER(NatEntry)), ("n_nat_entries", C.c_uint32),
                ("nat_port_ranges", C.POINTER(PortRange)), ("n_nat_port_ranges", C.c_uint32),
                ("nat_ranges", C.POINTER(NatRange)), ("n_nat_ranges", C.c_uint32),
                ("portfw", C.POINTER(PortFwRule)), ("n_portfw", C.c_uint32),
                ("masq", C.POINTER(MasqExpose)), ("n_masq", C.c_uint32),
                ("masq_prefixes", C.POINTER(Prefix)), ("n_masq_prefixes", C.c_uint32),
                ("masq_claims", C.POINTER(MasqClaim)), ("n_masq_claims", C.c_uint32),
                ("masq_config_tag", C.c_uint64), ("masq_randomize", C.c_uint32), ("pad1", C.c_uint32),
                ("masq_seed", C.c_uint64)]


STRUCTS = dict(dp_ipaddr_t=IpAddr, dp_prefix_t=Prefix, dp_fib_t=Fib, dp_vni_fib_t=VniFib,
               dp_instr_t=Instr, dp_fib_entry_t=FibEntry, dp_route_nh_t=RouteNh,
               dp_route_t=Route, dp_iface_t=Iface, dp_adjacency_t=Adjacency, dp_rule_t=Rule,
               dp_acl_default_t=AclDefault, dp_nat_table_t=NatTable, dp_nat_entry_t=NatEntry,
               dp_port_range_t=PortRange, dp_nat_range_t=NatRange, dp_portfw_rule_t=PortFwRule,
               dp_masq_expose_t=MasqExpose, dp_masq_claim_t=MasqClaim, dp_tables_desc_t=TablesDesc)

# every symbol include/dpgpu.h declares
GPU_SYMBOLS = ["dp_abi_version", "dp_ctx_create", "dp_ctx_destroy", "dp_tables_publish",
               "dp_tables_genid", "dp_process_burst", "dp_process_burst_device",
               "dp_process_burst_sharded", "dp_ctx_synchronize", "dp_tables_device_bytes",
               "dp_last_error", "dp_ctx_set_option", "dp_flow_table_create",
               "dp_flow_table_destroy", "dp_flow_table_set_capacity", "dp_flow_insert",
               "dp_flow_insert_pair", "dp_flow_lookup", "dp_flow_get", "dp_flow_remove",
               "dp_flow_invalidate", "dp_flow_set_status", "dp_flow_sweep", "dp_flow_count",
               "dp_ctx_attach_flow_table", "dp_mbuf_burst_in", "dp_mbuf_burst_out",
               "dp_process_mbufs", "dp_acl_classify", "dp_acl_classify_device",
               "dp_acl_key_from_match", "dp_acl_classify_match", "dp_ff_classify",
               "dp_ff_classify_device", "dp_ff_key_from_match", "dp_ff_classify_match"]
# dp_acl_key_t / dp_acl_result_t (the ACL classifier alone)
ACL_KEY = np.dtype([("src_vni", "<u4"), ("dst_vni", "<u4"), ("family", "u1"), ("proto", "u1"),
                    ("sport", "<u2"), ("dport", "<u2"), ("pad", "u1", 2), ("src", "u1", 16),
                    ("dst", "u1", 16)])
# the reference's AclKey bytes (MatchKey::as_key_into; dp_acl_key_from_match)
ACL_MATCH_KEY_V4, ACL_MATCH_KEY_V6 = 21, 45
ACL_RESULT = np.dtype([("rule", "<u4"), ("action", "u1"), ("scope", "u1"), ("acl", "u1"), ("pad", "u1")])
# dp_ff_input_t / dp_ff_result_t (the flow-filter classifier alone:
# LookupInput / LookupResult, flow-filter/src/context/tables.rs:70-97)
FF_INPUT = np.dtype([("src_vni", "<u4"), ("dst_vni", "<u4"), ("src_family", "u1"), ("dst_family", "u1"),
                     ("proto", "u1"), ("gate", "u1"), ("sport", "<u2"), ("dport", "<u2"), ("pad", "u1", 4),
                     ("src", "u1", 16), ("dst", "u1", 16)])
FF_RESULT = np.dtype([("outcome", "u1"), ("dst_nat", "u1"), ("src_nat", "u1"), ("pad", "u1"),
                      ("dst_vni", "<u4")])
FF_DESTINATION_MISS, FF_SOURCE_MISS, FF_ROUTE = 0, 1, 2
FF_REMOTE, FF_LOCAL = 1, 2
# the reference's RemoteKey / LocalKey bytes (MatchKey::as_key_into; dp_ff_key_from_match)
FF_REMOTE_KEY_V4, FF_REMOTE_KEY_V6, FF_LOCAL_KEY_V4, FF_LOCAL_KEY_V6 = 15, 27, 16, 28
NP_STRUCTS = dict(dp_flow_key_t=FLOW_KEY, dp_flow_t=FLOW, dp_flow_info_t=FLOW_INFO, dp_acl_key_t=ACL_KEY,
                  dp_acl_result_t=ACL_RESULT, dp_ff_input_t=FF_INPUT, dp_ff_result_t=FF_RESULT)


class MbufLayout(C.Structure):
    """dp_mbuf_layout_t: byte offsets of the rte_mbuf fields the DPDK glue uses."""
    _fields_ = [("buf_addr", C.c_uint16), ("data_off", C.c_uint16), ("nb_segs", C.c_uint16),
                ("port", C.c_uint16), ("pkt_len", C.c_uint16), ("data_len", C.c_uint16),
                ("buf_len", C.c_uint16), ("pad", C.c_uint16)]


MBUF_LAYOUT_DPDK = MbufLayout(0, 16, 20, 22, 36, 40, 54, 0)  # DP_MBUF_LAYOUT_DPDK

# dp_ctx_set_option (include/dpgpu.h)
OPT_HOST_PATH = 1
OPT_CLOCK = 2
HOST_AUTO, HOST_COPY, HOST_ZERO_COPY = 0, 1, 2

_VP = C.c_void_p
_U8P = C.POINTER(C.c_uint8)


def _load(path: str) -> C.CDLL:
    if not os.path.exists(path):
        raise RuntimeError(f"native library missing: {path} (run __graft_entry__.build())")
    return C.CDLL(path)


def _one_hip_runtime() -> None:
    """One HIP runtime per process (dp_ctx_create refuses two).
    PyTorch bundles its own libamdhip64 / libhsa-runtime64 and its libraries
    ask for them by the unversioned name, which libdpgpu.so's
    libamdhip64.so.7 (the ROCm runtime it was linked against) does not
    answer: with libdpgpu.so loaded first, a later `import torch` would map a
    second runtime beside it.  So where PyTorch is installed its runtime is
    loaded first; libdpgpu.so's libamdhip64.so.7 then resolves to it by its
    soname, and PyTorch finds the same files already mapped.  Nothing is
    imported, nothing touches the GPU."""
    if "torch" in sys.modules:
        return  # (its runtime is mapped already; libdpgpu.so resolves to it)
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.submodule_search_locations:
        return
    d = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        if not os.path.exists(os.path.join(d, name)):
            return
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        C.CDLL(os.path.join(d, name), mode=C.RTLD_GLOBAL)


_gpu = None


def gpu_lib() -> C.CDLL:
    """The product library (HIP).  Raises if it is not built."""
    global _gpu
    if _gpu is None:
        # DPGPU_LIB selects a diagnostic build (e.g. lib/libdpgpu_timing.so)
        if not os.environ.get("DPGPU_NO_RUNTIME_PRELOAD"):  # (hip_runtimes_diag.py's two-runtime leg)
            _one_hip_runtime()
        lib = _load(os.environ.get("DPGPU_LIB") or os.path.join(LIB_DIR, "libdpgpu.so"))
        lib.dp_abi_version.restype = C.c_uint32
        lib.dp_ctx_create.argtypes = [C.c_int, C.POINTER(_VP)]
        lib.dp_ctx_destroy.argtypes = [_VP]
        lib.dp_tables_publish.argtypes = [_VP, C.POINTER(TablesDesc)]
        lib.dp_tables_genid.argtypes = [_VP]
        lib.dp_tables_genid.restype = C.c_int64
        lib.dp_process_burst.argtypes = [_VP, _VP, C.c_uint64, _VP, _VP, _VP, C.c_uint32, _VP]
        lib.dp_process_burst_device.argtypes = [_VP, _VP, C.c_uint64, _VP, _VP, _VP,
                                                C.c_uint32, _VP, _VP]
        lib.dp_process_burst_sharded.argtypes = [C.POINTER(_VP), C.c_uint32, _VP, C.c_uint64,
                                                 _VP, _VP, _VP, C.c_uint32, _VP]
        lib.dp_ctx_synchronize.argtypes = [_VP]
        lib.dp_tables_device_bytes.argtypes = [_VP]
        lib.dp_tables_device_bytes.restype = C.c_uint64
        lib.dp_last_error.restype = C.c_char_p
        lib.dp_ctx_set_option.argtypes = [_VP, C.c_int, C.c_int64]
        lib.dp_flow_table_create.argtypes = [C.c_int, C.c_uint64, C.POINTER(_VP)]
        lib.dp_flow_table_destroy.argtypes = [_VP]
        lib.dp_flow_table_set_capacity.argtypes = [_VP, C.c_uint64]
        lib.dp_flow_insert.argtypes = [_VP, _VP, C.c_uint32, _VP, _VP]
        lib.dp_flow_insert_pair.argtypes = [_VP, _VP, _VP, _VP, _VP]
        lib.dp_flow_lookup.argtypes = [_VP, _VP, C.c_uint32, _VP]
        lib.dp_flow_get.argtypes = [_VP, _VP, C.c_uint32, _VP]
        lib.dp_flow_remove.argtypes = [_VP, _VP, C.c_uint32, _VP]
        lib.dp_flow_invalidate.argtypes = [_VP, _VP, C.c_uint32]
        lib.dp_flow_set_status.argtypes = [_VP, C.c_uint64, C.c_uint32]
        lib.dp_flow_sweep.argtypes = [_VP, C.c_uint64, _VP]
        lib.dp_flow_count.argtypes = [_VP, _VP, _VP]
        lib.dp_ctx_attach_flow_table.argtypes = [_VP, _VP]
        lib.dp_mbuf_burst_in.argtypes = [_VP, C.c_uint64, _VP, C.c_uint32, C.POINTER(MbufLayout),
                                         _VP, C.c_uint32, _VP]
        lib.dp_mbuf_burst_out.argtypes = [_VP, C.c_uint32, C.POINTER(MbufLayout), _VP, _VP]
        lib.dp_process_mbufs.argtypes = [_VP, _VP, C.c_uint64, _VP, C.c_uint32,
                                         C.POINTER(MbufLayout), _VP, C.c_uint32, _VP, _VP, _VP]
        lib.dp_acl_classify.argtypes = [_VP, _VP, _VP, C.c_uint32]
        lib.dp_acl_classify_device.argtypes = [_VP, _VP, _VP, C.c_uint32, _VP]
        lib.dp_acl_key_from_match.argtypes = [_VP, C.c_uint32, C.c_uint32, C.c_uint32, _VP]
        lib.dp_acl_classify_match.argtypes = [_VP, _VP, C.c_uint32, C.c_uint32, C.c_uint32, _VP]
        lib.dp_ff_classify.argtypes = [_VP, _VP, _VP, C.c_uint32]
        lib.dp_ff_classify_device.argtypes = [_VP, _VP, _VP, C.c_uint32, _VP]
        lib.dp_ff_key_from_match.argtypes = [C.c_int, _VP, C.c_uint32, C.c_uint32, C.c_uint32, _VP]
        lib.dp_ff_classify_match.argtypes = [_VP, C.c_int, _VP, C.c_uint32, C.c_uint32, C.c_uint32, _VP]
        lib.dpd_debug_classify_copies.argtypes = [C.c_int]
        lib.dpd_debug_hip_runtimes.restype = C.c_int
        lib.dpf_debug_nat_sequential.argtypes = [C.c_int]
        lib.dpf_debug_nat_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32]
        lib.dpf_debug_nat_counters.restype = C.c_int
        lib.dpf_debug_flows_full.argtypes = [C.c_int]
        lib.dpf_debug_last_lean.restype = C.c_int
        lib.dpf_debug_no_ctx.argtypes = [C.c_int]
        lib.dpf_debug_replay_fork.argtypes = [C.c_int]
        if lib.dp_abi_version() != ABI_VERSION:
            raise RuntimeError("libdpgpu.so ABI version mismatch")
        _gpu = lib
    return _gpu


_work = None


class WorkloadConfig(C.Structure):
    _fields_ = [("config", C.c_uint32), ("n_packets", C.c_uint32), ("seed", C.c_uint64),
                ("n_routes_v4", C.c_uint32), ("n_routes_v6", C.c_uint32),
                ("n_acl", C.c_uint32), ("n_nat", C.c_uint32), ("n_vni", C.c_uint32),
                ("tcp_percent", C.c_uint32), ("layout", C.c_uint32)]


def work_lib() -> C.CDLL:
    """Synthetic workload generator (harness library, host only)."""
    global _work
    if _work is None:
        lib = _load(os.path.join(LIB_DIR, "libdpwork.so"))
        lib.dpw_build.argtypes = [C.POINTER(WorkloadConfig), C.POINTER(_VP)]
        lib.dpw_free.argtypes = [_VP]
        lib.dpw_tables.argtypes = [_VP]
        lib.dpw_tables.restype = C.POINTER(TablesDesc)
        lib.dpw_buf.argtypes = [_VP]
        lib.dpw_buf.restype = _U8P
        lib.dpw_buf_bytes.argtypes = [_VP]
        lib.dpw_buf_bytes.restype = C.c_uint64
        lib.dpw_in.argtypes = [_VP]
        lib.dpw_in.restype = _VP
        lib.dpw_n.argtypes = [_VP]
        lib.dpw_n.restype = C.c_uint32
        lib.dpw_frame_bytes.argtypes = [_VP]
        lib.dpw_frame_bytes.restype = C.c_uint64
        lib.dpw_sizeof.argtypes = [C.c_char_p]
        lib.dpw_sizeof.restype = C.c_uint32
        _work = lib
    return _work


def check(rc: int, what: str, lib=None) -> None:
    if rc != 0:
        msg = ""
        if lib is not None and hasattr(lib, "dp_last_error"):
            msg = (lib.dp_last_error() or b"").decode(errors="replace")
        raise RuntimeError(f"{what} failed: rc={rc} {msg}")
