// etcd_quorum.hpp — C++ host mirror of etcd's raft/quorum + raft/tracker API
// (reference: /root/reference/raft/quorum/*.go, raft/tracker/tracker.go),
// layered on the C ABI in etcd_quorum.h.  Same names, argument meaning and
// results as the Go package; every decision runs on the GPU through the batch
// kernels (per-group methods evaluate a batch of one; the *Batch functions
// evaluate many groups in one launch).  There is no CPU decision path: a
// missing or failing device surfaces as etcd_amd::EngineError.
#pragma once

#include <stdint.h>

#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "etcd_quorum.h"

namespace etcd_amd {

// Error raised for any non-QE_OK status of the C ABI.
class EngineError : public std::runtime_error {
 public:
  EngineError(const std::string &fn, int status);
  int status;
};

namespace quorum {

// quorum.Index (raft/quorum/quorum.go:23-30); MaxUint64 prints as "∞".
using Index = uint64_t;
constexpr Index kIndexInf = UINT64_MAX;
std::string IndexString(Index i);

// quorum.VoteResult (raft/quorum/quorum.go:48-58).
enum class VoteResult : uint8_t { VotePending = 1, VoteLost = 2, VoteWon = 3 };
const char *VoteResultString(VoteResult r);  // voteresult_string.go

// quorum.AckedIndexer (raft/quorum/quorum.go:34-36).
class AckedIndexer {
 public:
  virtual ~AckedIndexer() = default;
  // AckedIndex(voterID) (idx Index, found bool)
  virtual bool AckedIndex(uint64_t voter_id, Index *idx) const = 0;
};

// mapAckIndexer (raft/quorum/quorum.go:38-43).
class MapAckIndexer : public AckedIndexer {
 public:
  MapAckIndexer() = default;
  MapAckIndexer(std::initializer_list<std::pair<const uint64_t, Index>> l) : m(l) {}
  bool AckedIndex(uint64_t voter_id, Index *idx) const override;
  std::map<uint64_t, Index> m;
};

using Votes = std::map<uint64_t, bool>;

// quorum.MajorityConfig (raft/quorum/majority.go:25).
class MajorityConfig {
 public:
  MajorityConfig() = default;
  MajorityConfig(std::initializer_list<uint64_t> l) : ids(l) {}
  explicit MajorityConfig(std::set<uint64_t> s) : ids(std::move(s)) {}
  size_t size() const { return ids.size(); }
  std::string String() const;          // majority.go:27-43
  std::vector<uint64_t> Slice() const;  // majority.go:103-111
  std::string Describe(const AckedIndexer &l) const;  // majority.go:45-101 (text)
  Index CommittedIndex(const AckedIndexer &l) const;  // majority.go:126-172
  quorum::VoteResult VoteResult(const Votes &votes) const;  // majority.go:178-210
  std::set<uint64_t> ids;
};

// quorum.JointConfig (raft/quorum/joint.go:19): [0] incoming, [1] outgoing.
class JointConfig {
 public:
  JointConfig() = default;
  JointConfig(MajorityConfig c0, MajorityConfig c1 = {}) : c{std::move(c0), std::move(c1)} {}
  std::string String() const;            // joint.go:21-26
  std::set<uint64_t> IDs() const;        // joint.go:30-38
  std::string Describe(const AckedIndexer &l) const;  // joint.go:40-44 (text)
  Index CommittedIndex(const AckedIndexer &l) const;        // joint.go:49-56
  quorum::VoteResult VoteResult(const Votes &votes) const;  // joint.go:61-75
  MajorityConfig c[2];
};

// Batch entry points: one GPU launch for all groups.
std::vector<Index> CommittedIndexBatch(const std::vector<JointConfig> &cfgs,
                                       const std::vector<const AckedIndexer *> &acked);
std::vector<VoteResult> VoteResultBatch(const std::vector<JointConfig> &cfgs,
                                        const std::vector<const Votes *> &votes);

}  // namespace quorum

namespace tracker {

enum StateType : uint8_t { StateProbe = 0, StateReplicate = 1, StateSnapshot = 2 };

// tracker.Progress fields on the quorum path (raft/tracker/progress.go:30-80).
struct Progress {
  uint64_t Match = 0, Next = 1;
  StateType State = StateProbe;
  uint64_t PendingSnapshot = 0;
  bool RecentActive = false;
  bool ProbeSent = false;
  bool IsLearner = false;
  std::string String() const;  // progress.go:214-236 (the fields kept here)
};

// tracker.Config (raft/tracker/tracker.go:27-78).
struct Config {
  quorum::JointConfig Voters;
  bool AutoLeave = false;
  std::set<uint64_t> Learners;
  std::set<uint64_t> LearnersNext;
  std::string String() const;  // tracker.go:80-94
};

struct TallyResult {
  int granted = 0, rejected = 0;
  quorum::VoteResult result = quorum::VoteResult::VotePending;
};

// tracker.ProgressTracker (raft/tracker/tracker.go:117-125).
class ProgressTracker : public Config {
 public:
  explicit ProgressTracker(int max_inflight = 256) : MaxInflight(max_inflight) {}
  bool IsSingleton() const;                      // tracker.go:156-160
  std::vector<uint64_t> VoterNodes() const;      // tracker.go:227-236
  std::vector<uint64_t> LearnerNodes() const;    // tracker.go:238-249
  void ResetVotes() { Votes.clear(); }           // tracker.go:252-254
  void RecordVote(uint64_t id, bool v);          // tracker.go:258-263
  uint64_t Committed() const;                    // tracker.go:177-179  (GPU)
  TallyResult TallyVotes() const;                // tracker.go:267-288  (GPU)
  bool QuorumActive() const;                     // tracker.go:215-225  (GPU)
  std::map<uint64_t, tracker::Progress> Progress;
  quorum::Votes Votes;
  int MaxInflight;
};

ProgressTracker MakeProgressTracker(int max_inflight);  // tracker.go:128-143

// Batch entry points over many trackers (one launch each).
std::vector<uint64_t> CommittedBatch(const std::vector<const ProgressTracker *> &pts);
std::vector<TallyResult> TallyVotesBatch(const std::vector<const ProgressTracker *> &pts);
std::vector<bool> QuorumActiveBatch(const std::vector<const ProgressTracker *> &pts);

}  // namespace tracker

namespace confchange {

// raftpb.ConfChangeType (raft/raftpb/raft.pb.go:224-227).
enum ConfChangeType : uint8_t {
  ConfChangeAddNode = 0,
  ConfChangeRemoveNode = 1,
  ConfChangeUpdateNode = 2,
  ConfChangeAddLearnerNode = 3,
};

struct ConfChangeSingle {
  ConfChangeType Type;
  uint64_t NodeID;
};

// (tracker.Config, tracker.ProgressMap, error) of the reference's Changer
// methods; Err is empty on success and holds the reference's error text
// otherwise.
struct Result {
  tracker::Config Config;
  std::map<uint64_t, tracker::Progress> Progress;
  std::string Err;
  bool ok() const { return Err.empty(); }
};

// confchange.Changer (raft/confchange/confchange.go:31-34).  Each method runs
// the change on the GPU (qe_confchange) for this one tracker; ChangeBatch
// runs one change per tracker in one launch.
class Changer {
 public:
  tracker::ProgressTracker Tracker;
  uint64_t LastIndex = 0;
  Result EnterJoint(bool autoLeave, const std::vector<ConfChangeSingle> &ccs) const;  // :49-76
  Result LeaveJoint() const;                                                        // :92-123
  Result Simple(const std::vector<ConfChangeSingle> &ccs) const;                    // :130-147
};

enum class Op : uint8_t { Simple = 1, EnterJoint = 2, EnterJointAutoLeave = 3, LeaveJoint = 4 };

std::vector<Result> ChangeBatch(const std::vector<const Changer *> &changers,
                                const std::vector<Op> &ops,
                                const std::vector<std::vector<ConfChangeSingle>> &ccs);

}  // namespace confchange
}  // namespace etcd_amd
