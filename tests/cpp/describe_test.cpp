// MajorityConfig::Describe / JointConfig::Describe of the C++ host API
// (include/etcd_quorum.hpp) against the text the reference's datadriven
// harness printed for every `committed` case (raft/quorum/testdata/*.txt;
// raft/quorum/majority.go:45-101, joint.go:40-44).  Host-only: no GPU call.
//   describe_test <repo root>
#include <stdio.h>

#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "etcd_quorum.hpp"

using namespace etcd_amd::quorum;

static std::vector<std::string> split(const std::string &s, char d) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == d) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  out.push_back(cur);
  return out;
}

int main(int argc, char **argv) {
  const std::string root = argc > 1 ? argv[1] : ".";
  std::ifstream in(root + "/tests/golden/describe_testdata.txt");
  if (!in) {
    printf("cannot open describe_testdata.txt\n");
    return 2;
  }
  std::string line;
  int n = 0, fails = 0;
  while (std::getline(in, line)) {
    // cfg|cfgj|acked|text (newlines as the two characters \n)
    const size_t p1 = line.find('|'), p2 = line.find('|', p1 + 1), p3 = line.find('|', p2 + 1);
    const std::string cfg = line.substr(0, p1), cfgj = line.substr(p1 + 1, p2 - p1 - 1);
    const std::string acked = line.substr(p2 + 1, p3 - p2 - 1);
    std::string want;
    const std::string esc = line.substr(p3 + 1);
    for (size_t i = 0; i < esc.size(); i++) {
      if (esc[i] == '\\' && i + 1 < esc.size() && esc[i + 1] == 'n') {
        want += '\n';
        i++;
      } else {
        want += esc[i];
      }
    }
    MajorityConfig c0, c1;
    for (const std::string &t : split(cfg, ','))
      if (!t.empty()) c0.ids.insert(std::stoull(t));
    for (const std::string &t : split(cfgj, ','))
      if (!t.empty()) c1.ids.insert(std::stoull(t));
    MapAckIndexer l;
    for (const std::string &t : split(acked, ',')) {
      if (t.empty()) continue;
      const size_t c = t.find(':');
      l.m[std::stoull(t.substr(0, c))] = std::stoull(t.substr(c + 1));
    }
    // a joint case renders the union of the halves (joint.go:40-44)
    const std::string got = JointConfig(c0, c1).Describe(l);
    if (got != want) {
      fails++;
      printf("MISMATCH cfg=%s cfgj=%s\n--- got\n%s--- want\n%s", cfg.c_str(), cfgj.c_str(),
             got.c_str(), want.c_str());
    }
    n++;
  }
  if (fails) return 1;
  printf("PASS: %d Describe cases\n", n);
  return 0;
}
