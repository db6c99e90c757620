// rtla_cli.cpp -- TLC-compatible command line over librtla.so.
//
// Replaces the reference's invocation (reference README.md:5, raft.cfg:1-15,
// .vscode/settings.json:5):
//     java tlc2.TLC [-workers W] [-coverage M] -config raft.cfg raft.tla
// with
//     rtla [-workers W] [-coverage M] [-gpus G] [-fpbits B] -config X.cfg SPEC.tla
//
// SPEC.tla is either the reference's raft.tla (sha256 checked: the semantics
// are compiled into the kernels, not parsed) or a wrapper module that
// EXTENDS raft and defines the model-checking operators of specs/MC.tla
// (StateConstraint, NoTwoLeaders, ElectionSafety, LogMatching); the raft.tla
// next to it is then hash-checked.  The cfg grammar is TLC's subset used by
// raft.cfg: SPECIFICATION, INVARIANT(S), CONSTRAINT(S), CONSTANT(S) with
// `Name = {a, b}` / `Name = "str"` / `Name = 3` / `Name = mv`, and \* / (* *)
// comments.  Output follows TLC's stdout lines.  Exit codes: 0 = no error,
// 12 = safety violation, 150/151 = spec/config errors, 255 = other errors
// (TLC's ExitStatus values as we understand them; not verified against a
// live TLC here).
#include <errno.h>
#include <signal.h>
#include <spawn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <filesystem>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/rtla.h"

extern char** environ;

static const char* RAFT_SHA256 = "683a120af29e3e5a805e291f756229d65914f8fb73dddd8c78bafef50a6f6b81";

// ------------------------------------------------------------- sha256 ----
namespace {
struct Sha256 {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  void block(const uint8_t* p) {
    static const uint32_t k[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)p[4 * i] << 24 | p[4 * i + 1] << 16 | p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
      uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + k[i] + w[i];
      uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  std::string digest(const std::string& data) {
    std::string m = data;
    uint64_t bits = (uint64_t)data.size() * 8;
    m.push_back((char)0x80);
    while (m.size() % 64 != 56) m.push_back(0);
    for (int i = 7; i >= 0; i--) m.push_back((char)(bits >> (8 * i)));
    for (size_t o = 0; o < m.size(); o += 64) block((const uint8_t*)m.data() + o);
    char out[65];
    for (int i = 0; i < 8; i++) snprintf(out + 8 * i, 9, "%08x", h[i]);
    return out;
  }
};

std::string read_file(const std::string& p, bool* ok) {
  std::ifstream f(p, std::ios::binary);
  *ok = (bool)f;
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

std::string now_str() {
  time_t t = time(nullptr);
  char b[64];
  strftime(b, sizeof b, "%Y-%m-%d %H:%M:%S", localtime(&t));
  return b;
}

// ------------------------------------------------------------ cfg parse ----
struct CfgFile {
  std::string specification;
  std::string symmetry;  // SYMMETRY operator name ("" = none)
  std::vector<std::string> invariants, constraints;
  std::map<std::string, std::vector<std::string>> sets;  // Name = {a, b}
  std::map<std::string, std::string> scalars;            // Name = "x" | 3 | mv
};

std::string strip_comments(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size();) {
    if (s.compare(i, 2, "\\*") == 0) {
      while (i < s.size() && s[i] != '\n') i++;
    } else if (s.compare(i, 2, "(*") == 0) {
      size_t j = s.find("*)", i + 2);
      i = j == std::string::npos ? s.size() : j + 2;
    } else {
      o.push_back(s[i++]);
    }
  }
  return o;
}

std::vector<std::string> tokenize(const std::string& s) {
  std::vector<std::string> t;
  for (size_t i = 0; i < s.size();) {
    char c = s[i];
    if (isspace((unsigned char)c)) { i++; continue; }
    if (c == '"') {
      size_t j = s.find('"', i + 1);
      if (j == std::string::npos) j = s.size() - 1;
      t.push_back(s.substr(i, j - i + 1));
      i = j + 1;
      continue;
    }
    if (c == '{' || c == '}' || c == ',' || c == '=') { t.push_back(std::string(1, c)); i++; continue; }
    if (c == '<' && s.compare(i, 2, "<-") == 0) { t.push_back("<-"); i += 2; continue; }
    size_t j = i;
    while (j < s.size() && !isspace((unsigned char)s[j]) && strchr("{},=\"", s[j]) == nullptr) j++;
    t.push_back(s.substr(i, j - i));
    i = j;
  }
  return t;
}

bool parse_cfg(const std::string& text, CfgFile* c, std::string* err) {
  auto t = tokenize(strip_comments(text));
  static const char* KW[] = {"SPECIFICATION", "INVARIANT", "INVARIANTS", "CONSTRAINT", "CONSTRAINTS",
                             "CONSTANT", "CONSTANTS", "INIT", "NEXT", "PROPERTY", "PROPERTIES",
                             "SYMMETRY", "VIEW", "CHECK_DEADLOCK", "ACTION_CONSTRAINT", "ACTION_CONSTRAINTS"};
  auto is_kw = [&](const std::string& s) {
    for (auto k : KW) if (s == k) return true;
    return false;
  };
  std::string mode;
  for (size_t i = 0; i < t.size();) {
    if (is_kw(t[i])) { mode = t[i++]; continue; }
    if (mode == "SPECIFICATION") { c->specification = t[i++]; continue; }
    if (mode == "INVARIANT" || mode == "INVARIANTS") { c->invariants.push_back(t[i++]); continue; }
    if (mode == "CONSTRAINT" || mode == "CONSTRAINTS") { c->constraints.push_back(t[i++]); continue; }
    if (mode == "CONSTANT" || mode == "CONSTANTS") {
      if (i + 2 >= t.size() || (t[i + 1] != "=" && t[i + 1] != "<-")) { *err = "bad CONSTANT near '" + t[i] + "'"; return false; }
      std::string name = t[i];
      i += 2;
      if (t[i] == "{") {
        std::vector<std::string> v;
        i++;
        while (i < t.size() && t[i] != "}") {
          if (t[i] != ",") v.push_back(t[i]);
          i++;
        }
        i++;
        c->sets[name] = v;
      } else {
        c->scalars[name] = t[i++];
      }
      continue;
    }
    if (mode == "SYMMETRY") { c->symmetry = t[i++]; continue; }
    if (mode == "VIEW" || mode == "PROPERTY" || mode == "PROPERTIES" || mode == "INIT" ||
        mode == "NEXT" || mode == "ACTION_CONSTRAINT" || mode == "ACTION_CONSTRAINTS") {
      *err = mode + " is not supported by this checker";
      return false;
    }
    if (mode == "CHECK_DEADLOCK") { i++; continue; }
    *err = "unexpected token '" + t[i] + "'";
    return false;
  }
  return true;
}

void usage() {
  fprintf(stderr,
          "usage: rtla [-workers W] [-coverage M] [-gpus G] [-fpbits B] [-membudget BYTES] [-dump-levels]\n"
          "            [-raft PATH/raft.tla] [-skip-spec-check]\n"
          "            [-checkpoint MINUTES] [-checkpointdir PREFIX] [-recover PREFIX]\n"
          "            -config FILE.cfg SPEC.tla\n");
}

std::string subst_names(const std::string& s, const std::vector<std::string>& servers,
                         const std::vector<std::string>& values) {
  // The row printer names servers s1..sN and values v1..vV; map them to the
  // cfg's model values.
  std::string o;
  for (size_t i = 0; i < s.size();) {
    char c = s[i];
    bool boundary = i == 0 || !(isalnum((unsigned char)s[i - 1]) || s[i - 1] == '_' || s[i - 1] == '"');
    if (boundary && (c == 's' || c == 'v') && i + 1 < s.size() && isdigit((unsigned char)s[i + 1]) &&
        (i + 2 >= s.size() || !isalnum((unsigned char)s[i + 2]))) {
      int k = s[i + 1] - '1';
      const auto& names = c == 's' ? servers : values;
      if (k >= 0 && k < (int)names.size()) { o += names[k]; i += 2; continue; }
    }
    o.push_back(c);
    i++;
  }
  return o;
}

// ---- -gpus N: one process per GPU.  The launcher (this process, which never
// touches a GPU) spawns N copies of itself with RTLA_RANK / RTLA_WORLD /
// RTLA_RENDEZVOUS in the environment and relays rank 0's exit status.  Rank 0
// creates the RCCL unique id and publishes it through the rendezvous file;
// every rank opens its context with it (rtla_open, one shard per rank).
int launch_ranks(int n, char** argv) {
  char dir[] = "/tmp/rtla-rdv-XXXXXX";
  if (!mkdtemp(dir)) { perror("mkdtemp"); return 255; }
  const std::string rdv = std::string(dir) + "/comm_id";
  std::vector<pid_t> pids;
  for (int r = 0; r < n; r++) {
    std::vector<std::string> env;
    for (char** e = environ; *e; e++)
      if (strncmp(*e, "RTLA_RANK=", 10) && strncmp(*e, "RTLA_WORLD=", 11) && strncmp(*e, "RTLA_RENDEZVOUS=", 16))
        env.push_back(*e);
    env.push_back("RTLA_RANK=" + std::to_string(r));
    env.push_back("RTLA_WORLD=" + std::to_string(n));
    env.push_back("RTLA_RENDEZVOUS=" + rdv);
    std::vector<char*> envp;
    for (auto& e : env) envp.push_back((char*)e.c_str());
    envp.push_back(nullptr);
    pid_t pid = 0;
    if (posix_spawn(&pid, "/proc/self/exe", nullptr, nullptr, argv, envp.data()) != 0) {
      perror("posix_spawn");
      return 255;
    }
    pids.push_back(pid);
  }
  // Reap ranks in whatever order they end.  A rank killed by a signal, or
  // ending with an error status other than the ones every rank reaches
  // together (0, 12 = invariant violated, 150/151 = spec/cfg errors), may
  // leave the others blocked in a collective: they get a grace period to end
  // on their own, then SIGTERM, then SIGKILL.  No rank is ever restarted.
  int code0 = 0, worst = 0, left = n;
  std::vector<bool> done(n, false);
  double abort_at = -1.0;  // monotonic seconds at which the survivors are terminated
  bool termed = false;
  auto now = []() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
  };
  while (left > 0) {
    int st = 0;
    const pid_t pid = waitpid(-1, &st, WNOHANG);
    if (pid > 0) {
      int r = 0;
      while (r < n && pids[r] != pid) r++;
      if (r == n || done[r]) continue;
      done[r] = true;
      left--;
      const int code = WIFEXITED(st) ? WEXITSTATUS(st) : 255;
      if (r == 0) code0 = code;
      else if (code && !worst) worst = code;
      const bool abnormal = !WIFEXITED(st) || (code != 0 && code != 12 && code != 150 && code != 151);
      if (abnormal && abort_at < 0 && left > 0) {
        fprintf(stderr, "rtla: rank %d ended abnormally (%s %d); stopping the other ranks in 10 s\n", r,
                WIFEXITED(st) ? "exit status" : "signal", WIFEXITED(st) ? code : WTERMSIG(st));
        abort_at = now() + 10.0;
      }
      continue;
    }
    if (pid < 0 && errno != EINTR) break;
    if (abort_at >= 0 && now() > abort_at) {
      for (int r = 0; r < n; r++)
        if (!done[r]) kill(pids[r], termed ? SIGKILL : SIGTERM);
      abort_at = now() + 5.0;
      termed = true;
    }
    usleep(20000);
  }
  (void)remove(rdv.c_str());
  (void)rmdir(dir);
  return code0 ? code0 : worst;
}

// This rank's RCCL id: rank 0 makes it (dry run: a fixed pattern, no GPU) and
// publishes it atomically (write + rename); the others wait for the file.
bool rendezvous(int rank, const char* path, bool dry, unsigned char id[128]) {
  if (rank == 0) {
    if (dry) {
      for (int k = 0; k < 128; k++) id[k] = (unsigned char)k;
    } else if (rtla_comm_id(id) != RTLA_OK) {
      return false;
    }
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f || fwrite(id, 1, 128, f) != 128) return false;
    if (fclose(f) != 0 || rename(tmp.c_str(), path) != 0) return false;
    return true;
  }
  for (int t = 0; t < 1200; t++) {  // up to 120 s
    FILE* f = fopen(path, "rb");
    if (f) {
      const bool ok = fread(id, 1, 128, f) == 128;
      fclose(f);
      if (ok) return true;
    }
    usleep(100000);
  }
  return false;
}

const char* COVER[] = {"Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest",
                       "AdvanceCommitIndex", "AppendEntries", "Receive", "DuplicateMessage", "DropMessage",
                       "UpdateTerm", "HandleRequestVoteRequest", "HandleRequestVoteResponse",
                       "HandleAppendEntriesRequest", "HandleAppendEntriesResponse", "DropStaleResponse"};
}  // namespace

int main(int argc, char** argv) {
  std::string cfgpath, spec;
  int coverage = 0, gpus = 1, fpbits = 0, workers = 1;
  bool dump_levels = false, skip_spec_check = false;
  std::string raft_opt;
  uint64_t membudget = 0;
  // TLC -checkpoint <minutes> / -recover <path> (the reference's .gitignore:2 states/ dir)
  double ckpt_minutes = 0;
  std::string ckpt_prefix = "states/ckpt", recover_prefix;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) { usage(); exit(255); }
      return argv[++i];
    };
    if (a == "-config") cfgpath = next();
    else if (a == "-coverage") coverage = atoi(next().c_str());
    else if (a == "-workers") { std::string w = next(); workers = w == "auto" ? 0 : atoi(w.c_str()); }
    else if (a == "-gpus") gpus = atoi(next().c_str());
    else if (a == "-fpbits") fpbits = atoi(next().c_str());
    else if (a == "-membudget") membudget = strtoull(next().c_str(), nullptr, 10);
    else if (a == "-dump-levels") dump_levels = true;
    else if (a == "-raft") raft_opt = next();
    else if (a == "-skip-spec-check") skip_spec_check = true;
    else if (a == "-checkpoint") ckpt_minutes = atof(next().c_str());
    else if (a == "-checkpointdir") ckpt_prefix = next();
    else if (a == "-recover") recover_prefix = next();
    else if (a == "-h" || a == "-help") { usage(); return 0; }
    else if (!a.empty() && a[0] == '-') { fprintf(stderr, "Error: unsupported option %s\n", a.c_str()); return 255; }
    else spec = a;
  }
  (void)workers;
  if (gpus < 1) { usage(); return 255; }
  if (gpus > 1 && !getenv("RTLA_RANK")) return launch_ranks(gpus, argv);
  const int rank = getenv("RTLA_RANK") ? atoi(getenv("RTLA_RANK")) : 0;
  const int world = getenv("RTLA_WORLD") ? atoi(getenv("RTLA_WORLD")) : 1;
  if (world != gpus || rank < 0 || rank >= world) {
    fprintf(stderr, "Error: rank %d of %d does not match -gpus %d\n", rank, world, gpus);
    return 255;
  }
  if (rank > 0 && !freopen("/dev/null", "w", stdout)) return 255;  // rank 0 prints TLC's output
  const bool dry = getenv("RTLA_CLI_DRYRUN") != nullptr;
  if (dry) {  // launch / rendezvous check only (CPU tests)
    unsigned char id[128];
    const char* rdv = getenv("RTLA_RENDEZVOUS");
    const bool ok = world == 1 || (rdv && rendezvous(rank, rdv, true, id));
    fprintf(stderr, "rtla rank %d of %d ready (id %02x%02x%02x%02x)\n", rank, world, ok ? id[0] : 255, ok ? id[1] : 255,
            ok ? id[2] : 255, ok ? id[3] : 255);
    return ok ? 0 : 255;
  }
  if (spec.empty()) { usage(); return 255; }
  if (cfgpath.empty()) {
    cfgpath = spec.substr(0, spec.size() > 4 && spec.compare(spec.size() - 4, 4, ".tla") == 0 ? spec.size() - 4 : spec.size()) + ".cfg";
  }
  printf("rtla (MI355X-native explicit-state checker for raft.tla), ABI %d\n", rtla_abi_version());
  // --- spec identity
  bool ok = false;
  std::string spec_text = read_file(spec, &ok);
  if (!ok) { printf("Error: cannot read %s\n", spec.c_str()); return 150; }
  std::string dir = spec.find('/') == std::string::npos ? "." : spec.substr(0, spec.rfind('/'));
  std::string base = spec.substr(spec.find('/') == std::string::npos ? 0 : spec.rfind('/') + 1);
  bool wrapper = base != "raft.tla";
  std::string raft_path = !raft_opt.empty() ? raft_opt : wrapper ? dir + "/raft.tla" : spec;
  std::string raft_text = raft_path == spec ? spec_text : read_file(raft_path, &ok);
  if (!ok && !skip_spec_check) {
    printf("Error: %s EXTENDS raft but %s is missing (give -raft PATH)\n", spec.c_str(), raft_path.c_str());
    return 150;
  }
  std::string h = skip_spec_check ? std::string(RAFT_SHA256) : Sha256().digest(raft_text);
  if (skip_spec_check) printf("Warning: -skip-spec-check: the identity of raft.tla is NOT verified\n");
  if (h != RAFT_SHA256) {
    printf("Error: %s has sha256 %s; this checker compiles the semantics of raft.tla %s only.\n",
           raft_path.c_str(), h.c_str(), RAFT_SHA256);
    return 150;
  }
  if (wrapper && spec_text.find("EXTENDS raft") == std::string::npos) {
    printf("Error: %s does not EXTEND raft\n", spec.c_str());
    return 150;
  }
  printf("Parsing file %s (raft.tla sha256 %.12s... verified)\n", spec.c_str(), h.c_str());
  // --- cfg
  std::string cfg_text = read_file(cfgpath, &ok);
  if (!ok) { printf("Error: cannot read config %s\n", cfgpath.c_str()); return 151; }
  CfgFile cf;
  std::string err;
  if (!parse_cfg(cfg_text, &cf, &err)) { printf("Error: %s: %s\n", cfgpath.c_str(), err.c_str()); return 151; }
  if (!cf.specification.empty() && cf.specification != "Spec") {
    printf("Error: SPECIFICATION %s: only Spec (raft.tla:469) is supported\n", cf.specification.c_str());
    return 151;
  }
  // Operators available: raft.tla defines none of the MC operators.
  auto defined = [&](const std::string& op) {
    if (!wrapper) return false;
    return op == "StateConstraint" || op == "NoTwoLeaders" || op == "ElectionSafety" || op == "LogMatching";
  };
  rtla_cfg c;
  memset(&c, 0, sizeof c);
  for (auto& inv : cf.invariants) {
    if (!defined(inv) || inv == "StateConstraint") {
      printf("Error: The invariant %s specified in the configuration file is not defined in the specification.\n",
             inv.c_str());
      return 150;
    }
    c.inv_mask |= inv == "NoTwoLeaders" ? RTLA_INV_NO_TWO_LEADERS : inv == "ElectionSafety" ? RTLA_INV_ELECTION_SAFETY
                                                                                        : RTLA_INV_LOG_MATCHING;
  }
  for (auto& k : cf.constraints) {
    if (k != "StateConstraint" || !defined(k)) {
      printf("Error: The constraint %s specified in the configuration file is not defined in the specification.\n",
             k.c_str());
      return 150;
    }
  }
  if (!cf.symmetry.empty()) {
    if (!wrapper || cf.symmetry != "Perms") {
      printf("Error: The symmetry %s specified in the configuration file is not defined in the specification.\n",
             cf.symmetry.c_str());
      return 150;
    }
    c.symmetry = 1;  // Perms == Permutations(Server) (specs/MC.tla)
  }
  if (cf.constraints.empty()) {
    printf("Error: no CONSTRAINT: raft.tla's state space is infinite (Timeout raft.tla:180 and Send raft.tla:106-110 "
           "are unbounded); add CONSTRAINT StateConstraint from specs/MC.tla.\n");
    return 151;
  }
  auto need_set = [&](const char* n) -> std::vector<std::string> {
    auto it = cf.sets.find(n);
    if (it == cf.sets.end()) { printf("Error: constant %s is not assigned a set in %s\n", n, cfgpath.c_str()); exit(151); }
    return it->second;
  };
  auto need_int = [&](const char* n) -> int {
    auto it = cf.scalars.find(n);
    if (it == cf.scalars.end()) { printf("Error: constant %s is not assigned in %s\n", n, cfgpath.c_str()); exit(151); }
    return atoi(it->second.c_str());
  };
  std::vector<std::string> servers = need_set("Server"), values = need_set("Value");
  c.n_server = (int)servers.size();
  c.n_value = (int)values.size();
  c.max_term = need_int("MaxTerm");
  c.max_log = need_int("MaxLogLen");
  c.max_copies = need_int("MaxCopies");
  c.max_msgs = cf.scalars.count("MaxInFlight") ? need_int("MaxInFlight") : 0;
  c.fpset_log2 = fpbits;
  c.mem_budget = membudget;
  static const char* strs[][2] = {{"Follower", "\"Follower\""}, {"Candidate", "\"Candidate\""},
                                  {"Leader", "\"Leader\""}, {"Nil", "\"Nil\""},
                                  {"RequestVoteRequest", "\"RequestVoteRequest\""},
                                  {"RequestVoteResponse", "\"RequestVoteResponse\""},
                                  {"AppendEntriesRequest", "\"AppendEntriesRequest\""},
                                  {"AppendEntriesResponse", "\"AppendEntriesResponse\""}};
  for (auto& p : strs) {
    auto it = cf.scalars.find(p[0]);
    if (it == cf.scalars.end() || it->second != p[1]) {
      printf("Error: constant %s must be bound to %s as in raft.cfg:8-15\n", p[0], p[1]);
      return 151;
    }
  }
  unsigned char comm_id[128];
  if (world > 1 && !rendezvous(rank, getenv("RTLA_RENDEZVOUS"), false, comm_id)) {
    fprintf(stderr, "Error: rank %d: RCCL rendezvous failed\n", rank);
    return 255;
  }
  rtla_ctx* ctx = nullptr;
  int st = rtla_open(&c, rank, world, world > 1 ? comm_id : nullptr, &ctx);
  if (st < 0) { printf("Error: %s\n", rtla_strerror(st)); return 255; }
  char info[1024];
  rtla_device_info(ctx, info, sizeof info);
  printf("Running breadth-first search Model-Checking with 128-bit fingerprints on %d GPU%s: %s\n", world,
         world > 1 ? "s (fingerprint-sharded, RCCL)" : "", info);
  printf("Starting... (%s)\n", now_str().c_str());
  printf("Computing initial states...\n");
  auto t0 = std::chrono::steady_clock::now();
  rtla_level_stats ls;
  memset(&ls, 0, sizeof ls);
  if (!recover_prefix.empty()) {
    st = rtla_recover(ctx, recover_prefix.c_str());
    if (st < 0) { printf("Error: cannot recover from %s: %s\n", recover_prefix.c_str(), rtla_strerror(st)); return 255; }
    printf("Recovering from checkpoint %s (completed).\n", recover_prefix.c_str());
  } else {
    st = rtla_init(ctx, &ls);
    printf("Finished computing initial states: 1 distinct state generated at %s.\n", now_str().c_str());
  }
  auto last_progress = t0, last_ckpt = t0;
  // With several ranks the checkpoint (a collective) must be decided alike
  // everywhere: the clock is then the job's device time (the per-level
  // maximum over ranks, identical on every rank), not this rank's wall clock.
  double dev_s = 0, dev_ckpt = 0;
  while (st == RTLA_OK) {
    st = rtla_step(ctx, &ls);
    if (st < 0) break;
    dev_s += ls.kernel_ms / 1e3;
    const double since = world > 1 ? dev_s - dev_ckpt
                                   : std::chrono::duration<double>(std::chrono::steady_clock::now() - last_ckpt).count();
    if (ckpt_minutes > 0 && st == RTLA_OK && since >= ckpt_minutes * 60) {
      dev_ckpt = dev_s;
      // in-process (no shell from a GPU-initialised process)
      std::error_code ec;
      if (ckpt_prefix.find('/') != std::string::npos)
        std::filesystem::create_directories(ckpt_prefix.substr(0, ckpt_prefix.rfind('/')), ec);
      printf("Checkpointing of run %s\n", ckpt_prefix.c_str());
      if (rtla_checkpoint(ctx, ckpt_prefix.c_str()) != RTLA_OK) printf("Warning: checkpoint failed\n");
      else printf("Checkpointing completed at (%s)\n", now_str().c_str());
      last_ckpt = std::chrono::steady_clock::now();
    }
    if (dump_levels)
      printf("  level %d: frontier %llu, new %llu, generated %llu, %.3f ms\n", ls.level,
             (unsigned long long)ls.frontier, (unsigned long long)ls.new_states, (unsigned long long)ls.generated,
             ls.seconds * 1e3);
    auto now = std::chrono::steady_clock::now();
    if (std::chrono::duration<double>(now - last_progress).count() >= 60.0 || st != RTLA_OK) {
      double mins = std::chrono::duration<double>(now - t0).count() / 60.0;
      printf("Progress(%d) at %s: %llu states generated (%.0f s/min), %llu distinct states found (%.0f ds/min), "
             "%llu states left on queue.\n",
             ls.level, now_str().c_str(), (unsigned long long)ls.generated_total, ls.generated_total / mins,
             (unsigned long long)ls.distinct_total, ls.distinct_total / mins,
             (unsigned long long)(st == RTLA_OK ? ls.new_states : 0));
      last_progress = now;
    }
  }
  double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  int exit_code = 0;
  if (st < 0) {
    printf("Error: %s\n", rtla_strerror(st));
    rtla_close(ctx);
    return 255;
  }
  int depth = 0;
  // depth = levels with new states; the last level returns new == 0 on DONE
  depth = st == RTLA_DONE ? ls.level - 1 : ls.level;
  if (st == RTLA_VIOLATION) {
    int32_t mask = 0, inm = 0;
    rtla_violation(ctx, &mask, &inm);
    const char* inv = mask & RTLA_INV_NO_TWO_LEADERS ? "NoTwoLeaders" : mask & RTLA_INV_ELECTION_SAFETY ? "ElectionSafety" : "LogMatching";
    printf("Error: Invariant %s is violated.\n", inv);
    printf("Error: The behavior up to this point is:\n");
    size_t n = 0;
    rtla_trace(ctx, nullptr, nullptr, 0, &n);
    int W = rtla_row_words(&c);
    std::vector<uint32_t> rows(n * W);
    std::vector<int32_t> labels(n);
    if (rtla_trace(ctx, rows.data(), labels.data(), n, &n) == RTLA_OK) {
      std::vector<char> buf(1 << 20);
      for (size_t k = 0; k < n; k++) {
        std::string lab = "Initial predicate";
        if (labels[k] >= 0) {
          char lb[256];
          rtla_action_name(&c, labels[k] & 0xffff, (labels[k] >> 16) & 0x7fff, lb, sizeof lb);
          lab = lb;
        }
        rtla_state_text(&c, rows.data() + k * W, buf.data(), buf.size());
        printf("State %zu: <%s>\n%s\n\n", k + 1, subst_names(lab, servers, values).c_str(),
               subst_names(buf.data(), servers, values).c_str());
      }
    }
    exit_code = 12;
  } else {
    printf("Model checking completed. No error has been found.\n");
    printf("  Estimates of the probability that TLC did not check all reachable states\n"
           "  because two distinct states had the same fingerprint:\n"
           "  calculated (optimistic):  val = %.1E\n",
           // TLC's formula (distinct x (generated - distinct) / 2^64), kept so
           // tools that parse this line read the quantity TLC reports
           (double)ls.distinct_total * (double)(ls.generated_total - ls.distinct_total) / 1.8446744073709552e19);
    // this checker's own estimate: the set stores 63 key bits (fp.b | 1) at
    // a slot chosen by fp.a; a probe compares each generated state with ~2
    // random keys at the loads used
    printf("  rtla 63-bit-key estimate:  val = %.1E\n", (double)ls.generated_total * 2.0 / 9.223372036854775808e18);
  }
  if (coverage) {
    uint64_t g[16], d[16];
    rtla_coverage(ctx, g, d, 16);
    printf("The coverage statistics at %s\n", now_str().c_str());
    for (int k = 0; k < 16; k++) {
      if (k == 7) continue;
      printf("<%s of module raft>: %llu:%llu\n", COVER[k], (unsigned long long)d[k], (unsigned long long)g[k]);
    }
    printf("End of statistics.\n");
  }
  printf("%llu states generated, %llu distinct states found, 0 states left on queue.\n",
         (unsigned long long)ls.generated_total, (unsigned long long)ls.distinct_total);
  printf("The depth of the complete state graph search is %d.\n", depth);
  printf("Finished in %.2fs at (%s)\n", secs, now_str().c_str());
  rtla_close(ctx);
  return exit_code;
}
