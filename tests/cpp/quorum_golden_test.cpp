// quorum_golden_test.cpp — the reference's TestDataDriven
// (raft/quorum/datadriven_test.go:36-250) and TestLeaderElectionInOneRoundRPC
// (raft/raft_paper_test.go:192-232) restated against the C++ host API
// (include/etcd_quorum.hpp), i.e. through the GPU kernels.  Reads the golden
// fixtures extracted into tests/golden/ by tests/golden/make_golden.py.
//
//   quorum_golden_test <repo-root>        exit 0 and "PASS" on success
#include <stdio.h>
#include <stdlib.h>

#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "etcd_quorum.hpp"

using namespace etcd_amd;
using quorum::Index;
using quorum::JointConfig;
using quorum::MajorityConfig;
using quorum::MapAckIndexer;
using quorum::VoteResult;

static int failures = 0;
#define EXPECT(cond, msg)                                        \
  do {                                                           \
    if (!(cond)) {                                               \
      std::cerr << "FAIL: " << msg << " (" #cond ")" << std::endl; \
      failures++;                                                \
    }                                                            \
  } while (0)

struct Case {
  std::string cmd, source;
  bool joint = false;
  uint64_t expect = 0;
  std::vector<uint64_t> cfg, cfgj;
  MapAckIndexer acked;
  quorum::Votes votes;
};

static std::vector<std::string> split(const std::string &s, char c) {
  std::vector<std::string> out;
  std::string cur;
  for (char ch : s) {
    if (ch == c) {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur += ch;
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

static std::string field(const std::string &tok, const char *key) {
  const std::string k = std::string(key) + "=";
  return tok.compare(0, k.size(), k) == 0 ? tok.substr(k.size()) : std::string();
}

static std::vector<Case> load_cases(const std::string &path) {
  std::ifstream in(path);
  std::vector<Case> cases;
  std::string line;
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    std::istringstream ss(line);
    Case c;
    int joint;
    std::string tcfg, tcfgj, tacked, tvotes;
    ss >> c.cmd >> joint >> c.expect >> tcfg >> tcfgj >> tacked >> tvotes >> c.source;
    c.joint = joint != 0;
    for (auto &x : split(field(tcfg, "cfg"), ',')) c.cfg.push_back(std::stoull(x));
    for (auto &x : split(field(tcfgj, "cfgj"), ',')) c.cfgj.push_back(std::stoull(x));
    for (auto &kv : split(field(tacked, "acked"), ',')) {
      auto p = split(kv, ':');
      c.acked.m[std::stoull(p[0])] = std::stoull(p[1]);
    }
    for (auto &kv : split(field(tvotes, "votes"), ',')) {
      auto p = split(kv, ':');
      c.votes[std::stoull(p[0])] = p[1] == "1";
    }
    cases.push_back(c);
  }
  return cases;
}

static MajorityConfig mc(const std::vector<uint64_t> &ids) {
  return MajorityConfig(std::set<uint64_t>(ids.begin(), ids.end()));
}

int main(int argc, char **argv) {
  const std::string root = argc > 1 ? argv[1] : ".";
  auto cases = load_cases(root + "/tests/golden/quorum_testdata.txt");
  EXPECT(cases.size() == 127, "127 datadriven cases");

  // --- per-case, as datadriven_test.go runs them -----------------------
  for (const Case &c : cases) {
    const MajorityConfig c0 = mc(c.cfg), c1 = mc(c.cfgj);
    if (c.cmd == "committed") {
      if (!c.joint) {
        const Index idx = c0.CommittedIndex(c.acked);
        EXPECT(idx == c.expect, c.source << ": " << quorum::IndexString(idx));
        // zero-joint and self-joint quorums (datadriven_test.go:179-185)
        EXPECT(JointConfig(c0, MajorityConfig()).CommittedIndex(c.acked) == idx, c.source);
        EXPECT(JointConfig(c0, c0).CommittedIndex(c.acked) == idx, c.source);
        // lowering a non-deciding voter does not change the result (:186-213)
        for (uint64_t id : c0.ids) {
          Index iidx = 0;
          const bool found = c.acked.AckedIndex(id, &iidx);
          if (found && idx > iidx && iidx > 0) {
            for (Index low : {iidx - 1, Index(0)}) {
              MapAckIndexer lo;
              for (uint64_t j : c0.ids) {
                Index x;
                if (j == id) lo.m[j] = low;
                else if (c.acked.AckedIndex(j, &x)) lo.m[j] = x;
              }
              EXPECT(c0.CommittedIndex(lo) == idx, c.source << " overlaying " << id);
            }
          }
        }
      } else {
        const JointConfig cc(c0, c1);
        const Index idx = cc.CommittedIndex(c.acked);
        EXPECT(idx == c.expect, c.source << ": " << quorum::IndexString(idx));
        EXPECT(JointConfig(c1, c0).CommittedIndex(c.acked) == idx, c.source << " symmetry");
      }
    } else {
      VoteResult r;
      if (!c.joint) {
        r = c0.VoteResult(c.votes);
      } else {
        r = JointConfig(c0, c1).VoteResult(c.votes);
        EXPECT(JointConfig(c1, c0).VoteResult(c.votes) == r, c.source << " symmetry");
      }
      EXPECT(static_cast<uint64_t>(r) == c.expect, c.source << ": " << quorum::VoteResultString(r));
    }
  }

  // --- the same cases as two batched launches ----------------------------
  std::vector<JointConfig> cc, vc;
  std::vector<const quorum::AckedIndexer *> acks;
  std::vector<const quorum::Votes *> votes;
  std::vector<uint64_t> want_c, want_v;
  for (const Case &c : cases) {
    if (c.cmd == "committed") {
      cc.emplace_back(mc(c.cfg), mc(c.cfgj));
      acks.push_back(&c.acked);
      want_c.push_back(c.expect);
    } else {
      vc.emplace_back(mc(c.cfg), mc(c.cfgj));
      votes.push_back(&c.votes);
      want_v.push_back(c.expect);
    }
  }
  auto got_c = quorum::CommittedIndexBatch(cc, acks);
  auto got_v = quorum::VoteResultBatch(vc, votes);
  for (size_t i = 0; i < got_c.size(); i++) EXPECT(got_c[i] == want_c[i], "batch committed " << i);
  for (size_t i = 0; i < got_v.size(); i++)
    EXPECT(static_cast<uint64_t>(got_v[i]) == want_v[i], "batch vote " << i);

  // --- TestLeaderElectionInOneRoundRPC via ProgressTracker ---------------
  std::ifstream el(root + "/tests/golden/election_table.txt");
  std::string line;
  int rows = 0;
  while (std::getline(el, line)) {
    if (line.empty()) continue;
    std::istringstream ss(line);
    int size;
    std::string want, tv;
    ss >> size >> want >> tv;
    tracker::ProgressTracker pt = tracker::MakeProgressTracker(256);
    for (int id = 1; id <= size; id++) {
      pt.Voters.c[0].ids.insert(id);
      pt.Progress[id] = tracker::Progress{};
    }
    pt.RecordVote(1, true);  // campaign self-vote (raft.go:803)
    std::string state = pt.TallyVotes().result == VoteResult::VoteWon ? "StateLeader" : "StateCandidate";
    for (auto &kv : split(field(tv, "votes"), ',')) {
      if (state != "StateCandidate") break;
      auto p = split(kv, ':');
      pt.RecordVote(std::stoull(p[0]), p[1] == "1");
      const auto t = pt.TallyVotes();
      if (t.result == VoteResult::VoteWon) state = "StateLeader";
      else if (t.result == VoteResult::VoteLost) state = "StateFollower";
    }
    EXPECT(state == want, "election row " << rows << ": " << state << " want " << want);
    rows++;
  }
  EXPECT(rows == 13, "13 election rows");

  // --- tracker: learners, first-vote-sticks, QuorumActive ------------------
  tracker::ProgressTracker pt(256);
  pt.Voters = JointConfig({1, 2, 3}, {3, 4, 5});
  pt.Learners = {6};
  const uint64_t m[] = {10, 7, 9, 3, 8, 100};
  for (uint64_t id = 1; id <= 6; id++) {
    tracker::Progress pr;
    pr.Match = m[id - 1];
    pr.IsLearner = id == 6;
    pr.RecentActive = id == 1 || id == 2 || id == 6;
    pt.Progress[id] = pr;
  }
  EXPECT(pt.Committed() == 8, "joint committed");
  pt.RecordVote(1, true);
  pt.RecordVote(1, false);
  pt.RecordVote(6, true);
  pt.RecordVote(4, false);
  auto t = pt.TallyVotes();
  EXPECT(t.granted == 1 && t.rejected == 1 && t.result == VoteResult::VotePending, "tally");
  EXPECT(!pt.QuorumActive(), "quorum inactive");
  pt.Progress[3].RecentActive = pt.Progress[5].RecentActive = true;
  EXPECT(pt.QuorumActive(), "quorum active");
  EXPECT(pt.Voters.String() == "(1 2 3)&&(3 4 5)", pt.Voters.String());
  EXPECT(quorum::IndexString(quorum::kIndexInf) == "∞", "inf string");

  if (failures) {
    std::cerr << failures << " failures" << std::endl;
    return 1;
  }
  std::cout << "PASS: " << cases.size() << " datadriven cases, " << rows
            << " election rows, tracker checks (C++ API on the GPU)" << std::endl;
  return 0;
}
