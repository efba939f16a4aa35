"""ctypes binding of the C ABI in include/etcd_quorum.h (libetcd_quorum.so).

This is the same surface a cgo binding would use.  The
library is the product: if it is missing this module raises at import time
-- there is no CPU fallback.
"""
import ctypes as C
import os

# torch must be imported BEFORE the library is dlopen'ed: torch ships its own
# libamdhip64.so.7 and device memory / streams come from torch, so the
# library's DT_NEEDED libamdhip64.so.7 has to bind to that same runtime
# instance (two HIP runtimes in one process do not see each other's devices).
import torch  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QE_LIB", os.path.join(_HERE, "lib", "libetcd_quorum.so"))

QE_ABI_VERSION = 8
QE_OK = 0
QE_EINVAL = -22
QE_ERANGE = -34
QE_EHIP = -1000
QE_ECOMM = -1001
QE_INDEX_INF = (1 << 64) - 1
QE_MAX_SLOTS = 16
QE_VOTE_PENDING, QE_VOTE_LOST, QE_VOTE_WON = 1, 2, 3
QE_STATE_FOLLOWER, QE_STATE_CANDIDATE, QE_STATE_LEADER, QE_STATE_PRE_CANDIDATE = 0, 1, 2, 3
QE_ELEC_PREVOTE, QE_ELEC_CHECK_QUORUM = 1, 2
QE_STATS_COUNTERS = 16
QE_STATS_SHARDS = 64
QE_STATS_WORDS = QE_STATS_COUNTERS * QE_STATS_SHARDS

STAT_NAMES = [
    "groups", "commit_inf", "commit_sum", "commit_zero", "vote_won", "vote_lost",
    "vote_pending", "granted", "rejected", "commit_advanced", "read_released", "elections",
    "leaders", "stepdowns", "invariant_violations", "checksum",
]

u64, u32, vp = C.c_uint64, C.c_uint32, C.c_void_p


class QeGroups(C.Structure):
    _fields_ = [
        ("num_groups", u64), ("group_offset", u64), ("num_slots", u32), ("reserved", u32),
        ("stride", u64), ("match", vp), ("inc_mask", vp), ("out_mask", vp),
        ("learner_mask", vp), ("voted", vp), ("granted", vp),
    ]


class QeOutputs(C.Structure):
    _fields_ = [("commit", vp), ("vote", vp), ("granted_count", vp), ("rejected_count", vp),
                ("stats", vp)]


class QeReplState(C.Structure):
    _fields_ = [
        ("num_groups", u64), ("group_offset", u64), ("num_slots", u32), ("reserved", u32),
        ("stride", u64), ("match", vp), ("next", vp), ("committed", vp), ("term_start", vp),
        ("last_index", vp), ("inc_mask", vp), ("out_mask", vp),
    ]


class QeReplMsgs(C.Structure):
    _fields_ = [("resp_index", vp), ("resp_mask", vp), ("read_acks", vp), ("read_ok", vp),
                ("commit_advanced", vp)]


class QeElectionState(C.Structure):
    _fields_ = [
        ("num_groups", u64), ("group_offset", u64), ("num_slots", u32), ("reserved", u32),
        ("term", vp), ("state", vp), ("voted", vp), ("granted", vp), ("self_slot", vp),
        ("inc_mask", vp), ("out_mask", vp), ("learner_mask", vp),
    ]


class QeElectionParams(C.Structure):
    _fields_ = [("seed", u64), ("step0", u64), ("steps", u32), ("p_drop_q16", u32),
                ("p_grant_q16", u32), ("flags", u32), ("p_active_q16", u32), ("reserved", u32),
                ("script_resp", vp), ("script_grant", vp), ("script_hup", vp),
                ("script_stride", u64)]


class QeGenParams(C.Structure):
    _fields_ = [
        ("seed", u64), ("group_offset", u64), ("dist", u32), ("p_absent_q16", u32),
        ("p_voted_q16", u32), ("p_granted_q16", u32), ("n_inc", u32), ("n_out", u32),
        ("mask_mode", u32), ("reserved", u32),
    ]


class QeConfStateCSR(C.Structure):
    _fields_ = [("num_groups", u64), ("voters", vp), ("voters_off", vp),
                ("voters_outgoing", vp), ("outgoing_off", vp), ("learners", vp),
                ("learners_off", vp), ("learners_next", vp), ("learners_next_off", vp),
                ("auto_leave", vp), ("perm", vp)]


class QeProgress(C.Structure):
    _fields_ = [
        ("num_groups", u64), ("group_offset", u64), ("num_slots", u32), ("inflight_cap", u32),
        ("stride", u64), ("match", vp), ("next", vp), ("pending_snapshot", vp), ("peer", vp),
        ("infl_lo", vp), ("infl_hi", vp), ("committed", vp),
        ("term_start", vp), ("first_index", vp), ("last_index", vp), ("log_runs", u32),
        ("reserved", u32), ("run_first", vp), ("run_term", vp), ("run_count", vp),
        ("inc_mask", vp), ("out_mask", vp),
        ("tracked", vp), ("self_slot", vp), ("lead_transferee", vp), ("snap_index", vp),
        ("max_ents", u32), ("reserved2", u32),
        ("read_acks", vp), ("read_head", vp), ("read_count", vp),  # ABI 5
        ("read_cap", u32), ("reserved3", u32), ("read_ovf", vp), ("read_keys", vp),  # ABI 7
        ("infl16", vp),  # ABI 8: the 16-bit Inflights form
    ]


class QePeerMsgs(C.Structure):
    _fields_ = [("type", vp), ("index", vp), ("reject_hint", vp), ("log_term", vp),
                ("sent", vp), ("bcast", vp), ("snap", vp), ("timeout_now", vp),
                ("msg_count", vp), ("msg_index", vp), ("bytes_requested", vp),
                ("read_ctx", vp), ("read_released", vp), ("term_commit", vp),  # ABI 5
                ("term_commit_index", vp)]


class QeProposals(C.Structure):  # ABI 6
    _fields_ = [("num_entries", vp), ("payload", vp), ("max_cc", u32), ("flags", u32),
                ("cc_stride", u64), ("cc_count", vp), ("cc_pos", vp), ("cc_leave", vp),
                ("cc_size", vp), ("applied", vp), ("pending_conf_index", vp),
                ("uncommitted_size", vp), ("max_uncommitted", u64), ("result", vp),
                ("cc_refused", vp), ("sent", vp), ("snap", vp), ("bytes_requested", vp)]


class QeSwitch(C.Structure):  # ABI 7
    _fields_ = [("switched", vp), ("result", vp), ("sent", vp), ("snap", vp),
                ("bytes_requested", vp)]


class QeLeader(C.Structure):  # ABI 7
    _fields_ = [("elected", vp), ("term", vp), ("flags", u32), ("reserved", u32),
                ("pending_conf_index", vp), ("uncommitted_size", vp), ("result", vp),
                ("sent", vp), ("snap", vp)]


QE_BL_NONE, QE_BL_LEADER, QE_BL_NOT_MEMBER, QE_BL_RUNS_FULL = 0, 1, 2, 3
QE_BL_BCAST = 1

QE_SW_NONE, QE_SW_REMOVED, QE_SW_NO_VOTERS, QE_SW_BCAST, QE_SW_PROBE = 0, 1, 2, 3, 4
QE_SW_OUTCOME, QE_SW_TRANSFER_ABORTED = 0x0F, 0x10

QE_PROP_NONE, QE_PROP_OK, QE_PROP_DROPPED_NOT_MEMBER, QE_PROP_DROPPED_TRANSFER, \
    QE_PROP_DROPPED_SIZE = 0, 1, 2, 3, 4
QE_PROP_BAD_CC = 5  # ABI 7: more conf-change entries than max_cc
QE_PROP_MAX_CC = 8
QE_PROP_APPEND_ONLY = 1

QE_PR_PROBE, QE_PR_REPLICATE, QE_PR_SNAPSHOT = 0, 1, 2
QE_PF_STATE, QE_PF_PROBE_SENT, QE_PF_RECENT_ACTIVE = 3, 4, 8
QE_PW_START_SHIFT, QE_PW_COUNT_SHIFT = 8, 16
QE_PF_RING_WIDE = 16
QE_PW_RING_MASK = 0xFF0000F0  # ring representation bits (ABI 4), not Progress state
QE_RING_EPOCH_MAX = 0x7FF


def QE_RING_PITCH(F):
    return (int(F) + 3) & ~3
QE_MSG_NONE, QE_MSG_APP_RESP, QE_MSG_APP_RESP_REJECT, QE_MSG_HEARTBEAT_RESP = 0, 1, 2, 3
QE_MSG_SNAP_STATUS, QE_MSG_SNAP_STATUS_REJECT, QE_MSG_UNREACHABLE = 4, 5, 6
QE_MSG_TRANSFER_LEADER = 7  # ABI 5
QE_READ_QUEUE = 4           # ABI 5: ReadIndex requests pending per group
QE_RI_NONE, QE_RI_RESPOND, QE_RI_POSTPONED, QE_RI_QUEUED, QE_RI_FULL = 0, 1, 2, 3, 4
QE_RI_DUPLICATE = 5         # ABI 7: the request's key is pending already
QE_READ_CAP_MAX = 255       # ABI 7: the longest queue (read_cap)
QE_RING16_MAX_F = 8         # ABI 8: the 16-bit Inflights form (infl16)
QE_RING16_MAX_SLOTS = 9
QE_MAX_INFLIGHT = 255
QE_MAX_LOG_RUNS = 16

QE_PACK_TOO_MANY_PEERS = 1
QE_PACK_LEARNER_IS_VOTER = 2
QE_PACK_LEARNER_NEXT_NOT_OUTGOING = 4
QE_PACK_ZERO_ID = 8


class QeConf(C.Structure):
    _fields_ = [
        ("num_groups", u64), ("num_slots", u32), ("reserved", u32), ("slot_ids", vp),
        ("inc_mask", vp), ("out_mask", vp), ("learner_mask", vp), ("learners_next_mask", vp),
        ("is_learner", vp), ("tracked", vp), ("auto_leave", vp),
    ]


class QeConfChanges(C.Structure):
    _fields_ = [
        ("max_changes", u32), ("reserved", u32), ("stride", u64), ("op", vp), ("count", vp),
        ("type", vp), ("node_id", vp), ("last_index", vp), ("result", vp),
        ("new_progress", vp),
    ]


QE_CC_ADD_NODE, QE_CC_REMOVE_NODE, QE_CC_UPDATE_NODE, QE_CC_ADD_LEARNER_NODE = 0, 1, 2, 3
QE_CC_OP_NONE, QE_CC_OP_SIMPLE, QE_CC_OP_ENTER_JOINT, QE_CC_OP_ENTER_JOINT_AUTO, \
    QE_CC_OP_LEAVE_JOINT = 0, 1, 2, 3, 4


# Every symbol include/etcd_quorum.h declares, with its prototype.
PROTOTYPES = {
    "qe_abi_version": (C.c_int, []),
    "qe_strerror": (C.c_char_p, [C.c_int]),
    "qe_mask_bytes": (C.c_size_t, [u32]),
    "qe_tune": (C.c_int, [C.c_char_p, C.c_int]),
    "qe_commit_vote": (C.c_int, [C.POINTER(QeGroups), C.POINTER(QeOutputs), vp]),
    "qe_committed_index": (C.c_int, [C.POINTER(QeGroups), vp, vp]),
    "qe_vote_result": (C.c_int, [C.POINTER(QeGroups), vp, vp]),
    "qe_quorum_active": (C.c_int, [C.POINTER(QeGroups), vp, vp, vp]),
    "qe_record_votes": (C.c_int, [u64, u32, vp, vp, vp, vp, vp]),
    "qe_replication_round": (C.c_int, [C.POINTER(QeReplState), C.POINTER(QeReplMsgs), vp, vp]),
    "qe_election_steps": (C.c_int, [C.POINTER(QeElectionState), C.POINTER(QeElectionParams),
                                    vp, vp]),
    "qe_stats_reduce": (C.c_int, [vp, vp, vp]),
    "qe_collect_scratch_bytes": (C.c_size_t, [u64]),
    "qe_collect": (C.c_int, [u64, u64, vp, vp, vp, vp, vp, vp, vp, vp]),
    "qe_gen_groups": (C.c_int, [C.POINTER(QeGroups), C.POINTER(QeGenParams), vp]),
    "qe_apply_append_resps": (C.c_int, [u64, u32, u64, vp, vp, u64, vp, vp, vp, vp, vp]),
    "qe_pack_confstate": (C.c_int, [C.POINTER(QeConfStateCSR), u32, vp, vp, vp, vp, vp, vp]),
    "qe_pack_conf": (C.c_int, [C.POINTER(QeConfStateCSR), C.POINTER(QeConf), vp, vp]),
    "qe_pack_order": (C.c_int, [C.POINTER(QeConfStateCSR), u32, vp, vp]),
    "qe_pack_match": (C.c_int, [u64, u32, vp, vp, vp, vp, vp, vp, u64, vp]),
    "qe_pack_votes": (C.c_int, [u64, u32, vp, vp, vp, vp, vp, vp, vp]),
    "qe_slot_lookup": (C.c_int, [u64, u32, vp, u64, vp, vp, vp]),
    "qe_pack_threads": (C.c_int, [C.c_int]),
    "qe_progress_step": (C.c_int, [C.POINTER(QeProgress), C.POINTER(QePeerMsgs), vp, vp]),
    "qe_progress_send": (C.c_int, [C.POINTER(QeProgress), vp, u32, vp, vp, vp]),
    "qe_check_quorum": (C.c_int, [C.POINTER(QeProgress), vp, vp, vp]),
    "qe_read_index": (C.c_int, [C.POINTER(QeProgress), vp, vp, u32, vp, vp, vp, vp]),
    "qe_propose": (C.c_int, [C.POINTER(QeProgress), C.POINTER(QeProposals), vp, vp]),
    "qe_heartbeat": (C.c_int, [C.POINTER(QeProgress), vp, vp, vp, vp]),
    "qe_switch_config": (C.c_int, [C.POINTER(QeProgress), C.POINTER(QeSwitch), vp, vp]),
    "qe_become_leader": (C.c_int, [C.POINTER(QeProgress), C.POINTER(QeLeader), vp, vp]),
    "qe_ring_pack": (C.c_int, [u64, u32, u32, u64, vp, vp, vp, vp]),
    "qe_ring_unpack": (C.c_int, [u64, u32, u32, u64, vp, vp, vp, vp]),
    "qe_ring_pack16": (C.c_int, [u64, u32, u32, u64, vp, vp, vp, vp, vp, vp]),
    "qe_ring_unpack16": (C.c_int, [u64, u32, u32, u64, vp, vp, vp, vp, vp, vp]),
    "qe_confchange": (C.c_int, [C.POINTER(QeConf), C.POINTER(QeConfChanges),
                                C.POINTER(QeProgress), vp]),
    "qe_comm_id_bytes": (C.c_size_t, []),
    "qe_comm_unique_id": (C.c_int, [vp]),
    "qe_comm_init": (C.c_int, [C.POINTER(vp), u32, u32, vp, C.c_int]),
    "qe_comm_init_timeout": (C.c_int, [C.POINTER(vp), u32, u32, vp, C.c_int, u32]),
    "qe_comm_destroy": (C.c_int, [vp]),
    "qe_comm_abort": (C.c_int, [vp]),
    "qe_allreduce_stats": (C.c_int, [vp, u32, vp, vp]),
}


class QuorumEngineError(RuntimeError):
    def __init__(self, fn, status):
        msg = _LIB.qe_strerror(status).decode() if _LIB is not None else str(status)
        super().__init__(f"{fn} failed: {status} ({msg})")
        self.status = status


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"etcd_amd: HIP library {LIB_PATH} is missing; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in PROTOTYPES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.qe_abi_version() != QE_ABI_VERSION:
        raise ImportError("etcd_amd: ABI version mismatch")
    return lib


_LIB = None
_LIB = _load()


def lib():
    return _LIB


def check(fn, status):
    if status != QE_OK:
        raise QuorumEngineError(fn, status)
    return status
