// confchange_golden_test.cpp — the reference's TestConfChangeDataDriven
// (raft/confchange/datadriven_test.go:29-98) restated against the C++ host
// API (etcd_amd::confchange::Changer, include/etcd_quorum.hpp), i.e. through
// the qe_confchange kernel.  Reads tests/golden/confchange_testdata.txt
// (extracted by tests/golden/make_golden.py).  A fresh tracker per file,
// LastIndex incremented after every command, the result committed only on
// success -- as the reference harness does.
//
//   confchange_golden_test <repo-root>      exit 0 and "PASS" on success
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "etcd_quorum.hpp"

using namespace etcd_amd;
using confchange::ConfChangeSingle;

static std::vector<std::string> split(const std::string &s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  out.push_back(cur);
  return out;
}

// datadriven_test.go:46-77: vN voter, lN learner, rN remove, uN update.
static std::vector<ConfChangeSingle> parse_ccs(const std::string &in) {
  std::vector<ConfChangeSingle> out;
  std::istringstream is(in);
  std::string tok;
  while (is >> tok) {
    ConfChangeSingle cc{confchange::ConfChangeAddNode, std::stoull(tok.substr(1))};
    switch (tok[0]) {
      case 'v': cc.Type = confchange::ConfChangeAddNode; break;
      case 'l': cc.Type = confchange::ConfChangeAddLearnerNode; break;
      case 'r': cc.Type = confchange::ConfChangeRemoveNode; break;
      case 'u': cc.Type = confchange::ConfChangeUpdateNode; break;
    }
    out.push_back(cc);
  }
  return out;
}

int main(int argc, char **argv) {
  const std::string root = argc > 1 ? argv[1] : ".";
  std::ifstream f(root + "/tests/golden/confchange_testdata.txt");
  std::string line, file;
  confchange::Changer c;
  int steps = 0, failures = 0;
  while (std::getline(f, line)) {
    const auto col = split(line, '\t');
    if (col.size() != 6) continue;
    if (col[0] != file) {  // each testdata file starts from an empty tracker
      file = col[0];
      c.Tracker = tracker::MakeProgressTracker(10);  // datadriven_test.go:31
      c.LastIndex = 0;
    }
    const auto ccs = parse_ccs(col[4]);
    confchange::Result r;
    if (col[2] == "simple") {
      r = c.Simple(ccs);
    } else if (col[2] == "enter-joint") {
      r = c.EnterJoint(col[3] == "autoleave=true", ccs);
    } else {
      r = c.LeaveJoint();
    }
    std::string got;
    if (!r.ok()) {
      got = r.Err;
    } else {
      c.Tracker.Voters = r.Config.Voters;
      c.Tracker.Learners = r.Config.Learners;
      c.Tracker.LearnersNext = r.Config.LearnersNext;
      c.Tracker.AutoLeave = r.Config.AutoLeave;
      c.Tracker.Progress = r.Progress;
      got = r.Config.String();
      for (const auto &kv : r.Progress)
        got += "|" + std::to_string(kv.first) + ": " + kv.second.String();
    }
    c.LastIndex++;
    steps++;
    if (got != col[5]) {
      std::cerr << "FAIL " << col[0] << ":" << col[1] << "\n  got:  " << got
                << "\n  want: " << col[5] << std::endl;
      failures++;
    }
  }
  if (steps != 58) {
    std::cerr << "FAIL: expected 58 steps, read " << steps << std::endl;
    failures++;
  }
  if (failures) return 1;
  std::cout << "PASS: " << steps << " confchange steps" << std::endl;
  return 0;
}
