"""CPU restatement of raft/confchange (the Changer) over ID-keyed sets and a
Progress map -- the reference's own data model.  TEST INFRASTRUCTURE ONLY:
it is the checker for the device kernel qe_confchange (tests/, never the
product path).

Pinned by the reference's golden vectors: all 58 steps of
raft/confchange/testdata/*.txt (TestConfChangeDataDriven,
raft/confchange/datadriven_test.go:29-98), replayed through this module and
compared as text (Config.String + ProgressMap.String, or the error text) in
tests/test_confchange_oracle.py.

Each function cites the reference lines it follows
(raft/confchange/confchange.go unless noted).
"""

# pb.ConfChangeType (raft/raftpb/raft.pb.go:224-227)
ADD_NODE, REMOVE_NODE, UPDATE_NODE, ADD_LEARNER_NODE = 0, 1, 2, 3

# per-group result codes of qe_confchange (include/etcd_quorum.h); the error
# strings are the reference's
OK = 0
ERR_INVARIANT = 1           # checkInvariants on the input (checkAndCopy :261-272)
ERR_ALREADY_JOINT = 2       # :54
ERR_ZERO_VOTER_JOINT = 3    # :60
ERR_NOT_JOINT = 4           # :97
ERR_SIMPLE_IN_JOINT = 5     # :136
ERR_BAD_TYPE = 6            # :170
ERR_REMOVED_ALL = 7         # :174
ERR_SIMPLE_MULTI = 8        # :143
ERR_INVARIANT_OUT = 9       # checkAndReturn on the result
ERR_NO_SLOT = 10            # slot model only: a new peer found no free slot

MESSAGES = {
    ERR_ALREADY_JOINT: "config is already joint",
    ERR_ZERO_VOTER_JOINT: "can't make a zero-voter config joint",
    ERR_NOT_JOINT: "can't leave a non-joint config",
    ERR_SIMPLE_IN_JOINT: "can't apply simple config change in joint config",
    ERR_REMOVED_ALL: "removed all voters",
    ERR_SIMPLE_MULTI: "more than one voter changed without entering joint config",
}

OP_NONE, OP_SIMPLE, OP_ENTER_JOINT, OP_ENTER_JOINT_AUTO, OP_LEAVE_JOINT = 0, 1, 2, 3, 4


class ChangeError(Exception):
    def __init__(self, code, text=None):
        super().__init__(text or MESSAGES.get(code, f"error {code}"))
        self.code = code


class Progress:
    """The Progress fields a configuration change touches
    (raft/tracker/progress.go:30-80; initProgress :244-262)."""

    __slots__ = ("match", "next", "state", "is_learner", "recent_active", "probe_sent",
                 "pending", "inflight")

    def __init__(self, next_, is_learner):
        self.match, self.next, self.state = 0, next_, "StateProbe"
        self.is_learner, self.recent_active, self.probe_sent = is_learner, True, False
        self.pending, self.inflight = 0, 0

    def copy(self):
        p = Progress(self.next, self.is_learner)
        for k in self.__slots__:
            setattr(p, k, getattr(self, k))
        return p

    def string(self):  # raft/tracker/progress.go:214-236 (fields used here)
        s = f"{self.state} match={self.match} next={self.next}"
        if self.is_learner:
            s += " learner"
        if self.state == "StateProbe" and self.probe_sent:
            s += " paused"
        if self.pending > 0:
            s += f" pendingSnap={self.pending}"
        if not self.recent_active:
            s += " inactive"
        return s


class Config:
    """tracker.Config (raft/tracker/tracker.go:28-78): Voters[0], Voters[1],
    Learners, LearnersNext (empty set == nil, as nilAwareAdd/Delete keep it),
    AutoLeave."""

    def __init__(self):
        self.inc, self.out, self.learners, self.lnext = set(), set(), set(), set()
        self.auto_leave = False

    def clone(self):
        c = Config()
        c.inc, c.out = set(self.inc), set(self.out)
        c.learners, c.lnext = set(self.learners), set(self.lnext)
        c.auto_leave = self.auto_leave
        return c

    def string(self):  # tracker.go:80-93, quorum/joint.go:21-26, majority.go:27-43
        def maj(s):
            return "(" + " ".join(str(i) for i in sorted(s)) + ")"
        v = maj(self.inc) + ("&&" + maj(self.out) if self.out else "")
        s = f"voters={v}"
        if self.learners:
            s += f" learners={maj(self.learners)}"
        if self.lnext:
            s += f" learners_next={maj(self.lnext)}"
        if self.auto_leave:
            s += " autoleave"
        return s


def progress_string(prs):  # raft/tracker/progress.go:242-255
    return [f"{i}: {prs[i].string()}" for i in sorted(prs)]


def check_invariants(cfg, prs):  # :186-241
    for ids in (cfg.inc | cfg.out, cfg.learners, cfg.lnext):
        for i in ids:
            if i not in prs:
                return f"no progress for {i}"
    for i in cfg.lnext:
        if i not in cfg.out:
            return f"{i} is in LearnersNext, but not Voters[1]"
        if prs[i].is_learner:
            return f"{i} is in LearnersNext, but is already marked as learner"
    for i in cfg.learners:
        if i in cfg.out:
            return f"{i} is in Learners and Voters[1]"
        if i in cfg.inc:
            return f"{i} is in Learners and Voters[0]"
        if not prs[i].is_learner:
            return f"{i} is in Learners, but is not marked as learner"
    if not cfg.out:
        # Voters[1] nil / LearnersNext nil hold by construction of the set model
        if cfg.lnext:
            return "cfg.LearnersNext must be nil when not joint"
        if cfg.auto_leave:
            return "AutoLeave must be false when not joint"
    return None


class Changer:
    """confchange.Changer{Tracker, LastIndex} (:31-34)."""

    def __init__(self, cfg=None, prs=None, last_index=0):
        self.cfg = cfg if cfg is not None else Config()
        self.prs = prs if prs is not None else {}
        self.last_index = last_index
        self.peak = 0  # most Progress entries held during the last run()

    def _check_and_copy(self):  # :252-262
        cfg = self.cfg.clone()
        prs = {i: p.copy() for i, p in self.prs.items()}
        err = check_invariants(cfg, prs)
        if err:
            raise ChangeError(ERR_INVARIANT, err)
        return cfg, prs

    @staticmethod
    def _check_and_return(cfg, prs):  # :266-271
        err = check_invariants(cfg, prs)
        if err:
            raise ChangeError(ERR_INVARIANT_OUT, err)
        return cfg, prs

    def enter_joint(self, auto_leave, ccs):  # :49-76
        cfg, prs = self._check_and_copy()
        if cfg.out:
            raise ChangeError(ERR_ALREADY_JOINT)
        if not cfg.inc:
            raise ChangeError(ERR_ZERO_VOTER_JOINT)
        cfg.out = set(cfg.inc)
        self._apply(cfg, prs, ccs)
        cfg.auto_leave = auto_leave
        return self._check_and_return(cfg, prs)

    def leave_joint(self):  # :92-123
        cfg, prs = self._check_and_copy()
        if not cfg.out:
            raise ChangeError(ERR_NOT_JOINT)
        for i in cfg.lnext:
            cfg.learners.add(i)
            prs[i].is_learner = True
        cfg.lnext = set()
        for i in cfg.out:
            if i not in cfg.inc and i not in cfg.learners:
                prs.pop(i, None)
        cfg.out = set()
        cfg.auto_leave = False
        return self._check_and_return(cfg, prs)

    def simple(self, ccs):  # :130-147
        cfg, prs = self._check_and_copy()
        if cfg.out:
            raise ChangeError(ERR_SIMPLE_IN_JOINT)
        self._apply(cfg, prs, ccs)
        if len(self.cfg.inc ^ cfg.inc) > 1:  # symdiff :384-401
            raise ChangeError(ERR_SIMPLE_MULTI)
        return self._check_and_return(cfg, prs)

    def _apply(self, cfg, prs, ccs):  # :152-177
        for typ, node in ccs:
            if node == 0:
                continue
            if typ == ADD_NODE:
                self._make_voter(cfg, prs, node)
            elif typ == ADD_LEARNER_NODE:
                self._make_learner(cfg, prs, node)
            elif typ == REMOVE_NODE:
                self._remove(cfg, prs, node)
            elif typ == UPDATE_NODE:
                pass
            else:
                raise ChangeError(ERR_BAD_TYPE, f"unexpected conf type {typ}")
        if not cfg.inc:
            raise ChangeError(ERR_REMOVED_ALL)

    def _make_voter(self, cfg, prs, i):  # :181-193
        pr = prs.get(i)
        if pr is None:
            self._init_progress(cfg, prs, i, False)
            return
        pr.is_learner = False
        cfg.learners.discard(i)
        cfg.lnext.discard(i)
        cfg.inc.add(i)

    def _make_learner(self, cfg, prs, i):  # :207-231
        pr = prs.get(i)
        if pr is None:
            self._init_progress(cfg, prs, i, True)
            return
        if pr.is_learner:
            return
        self._remove(cfg, prs, i)
        prs[i] = pr
        if i in cfg.out:
            cfg.lnext.add(i)
        else:
            pr.is_learner = True
            cfg.learners.add(i)

    def _remove(self, cfg, prs, i):  # :234-248
        if i not in prs:
            return
        cfg.inc.discard(i)
        cfg.learners.discard(i)
        cfg.lnext.discard(i)
        if i not in cfg.out:
            del prs[i]

    def _init_progress(self, cfg, prs, i, is_learner):  # :251-274
        if not is_learner:
            cfg.inc.add(i)
        else:
            cfg.learners.add(i)
        prs[i] = Progress(self.last_index, is_learner)
        self.peak = max(self.peak, len(prs))

    def run(self, op, ccs):
        """One qe_confchange op on this group; commits the result (as the
        datadriven harness does, datadriven_test.go:93-97) and returns the
        result code.  Changer.LastIndex is the caller's.  self.peak records
        the most Progress entries the change held at once (a slot-model
        caller runs out of slots exactly when it exceeds the slot count)."""
        self.peak = len(self.prs)
        try:
            if op == OP_NONE:
                return OK
            if op == OP_SIMPLE:
                cfg, prs = self.simple(ccs)
            elif op in (OP_ENTER_JOINT, OP_ENTER_JOINT_AUTO):
                cfg, prs = self.enter_joint(op == OP_ENTER_JOINT_AUTO, ccs)
            elif op == OP_LEAVE_JOINT:
                cfg, prs = self.leave_joint()
            else:
                raise ValueError(op)
        except ChangeError as e:
            return e.code
        self.cfg, self.prs = cfg, prs
        return OK


def parse_changes(text):
    """datadriven_test.go:46-77: vN voter, lN learner, rN remove, uN update."""
    kinds = {"v": ADD_NODE, "l": ADD_LEARNER_NODE, "r": REMOVE_NODE, "u": UPDATE_NODE}
    return [(kinds[t[0]], int(t[1:])) for t in text.split()]


def replay(steps):
    """Replays one testdata file; yields (step, output lines)."""
    c = Changer()
    for st in steps:
        ccs = parse_changes(st["input"])
        try:
            if st["cmd"] == "simple":
                cfg, prs = c.simple(ccs)
            elif st["cmd"] == "enter-joint":
                auto = "autoleave=true" in st["args"]
                cfg, prs = c.enter_joint(auto, ccs)
            else:
                if ccs:
                    raise ChangeError(-1, "this command takes no input")
                cfg, prs = c.leave_joint()
            c.cfg, c.prs = cfg, prs
            out = [cfg.string()] + progress_string(prs)
        except ChangeError as e:
            out = [str(e)]
        c.last_index += 1  # datadriven_test.go:41-43
        yield st, out
