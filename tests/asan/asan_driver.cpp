// Host-side sanitizer driver for the native data path (csrc/bpe.cpp, csrc/data.cpp, capi.cpp),
// built with -fsanitize=address,undefined by tests/test_asan_host.py. It replays the golden
// fixtures through the C ABI exactly as the DataLoader workers call it -- single and batched
// multithreaded BPE, BERT masking, FASTA windows -- plus a fork of the process holding the open
// handles (the workers' situation), and exits 0 only when every output matches.
//   asan_driver <bpe.json> <cases.txt> <fasta>
// cases.txt lines:  B <window> | <full ids...>     (BPE, raw window bytes without spaces)
//                   D <P> <row ids...>             (dataset-form ids of the preceding window)
//                   F <chr> <start> <end> <max_length> <pad> <expected window or ->
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <sstream>
#include <string>
#include <vector>

#include "dna_amd.h"

static int fails = 0;
#define CHECK(c, ...)                         \
  do {                                        \
    if (!(c)) {                               \
      fprintf(stderr, "FAIL: " __VA_ARGS__);  \
      fprintf(stderr, "\n");                  \
      ++fails;                                \
    }                                         \
  } while (0)

struct BpeCase {
  std::string win;
  std::vector<int> full;
  int P = 0;
  std::vector<int> ds;
};

int main(int argc, char** argv) {
  if (argc != 4) return 2;
  dna_bpe* bpe = dna_bpe_create(argv[1]);
  if (!bpe) { fprintf(stderr, "bpe: %s\n", dna_last_error()); return 3; }
  dna_fasta* fa = dna_fasta_open(argv[3]);
  if (!fa) { fprintf(stderr, "fasta: %s\n", dna_last_error()); return 3; }
  FILE* f = fopen(argv[2], "r");
  if (!f) return 3;
  std::vector<BpeCase> cases;
  char* line = nullptr;
  size_t cap = 0;
  int nf = 0;
  while (getline(&line, &cap, f) > 0) {
    std::istringstream in(line);
    std::string kind;
    in >> kind;
    if (kind == "B") {
      BpeCase c;
      std::string w, bar;
      in >> w;
      c.win = w == "-" ? std::string() : w;
      in >> bar;
      int id;
      while (in >> id) c.full.push_back(id);
      cases.push_back(c);
    } else if (kind == "D") {
      in >> cases.back().P;
      int id;
      while (in >> id) cases.back().ds.push_back(id);
    } else if (kind == "F") {
      std::string chr, want;
      long long s, e, ml;
      int pad;
      in >> chr >> s >> e >> ml >> pad >> want;
      if (want == "-") want.clear();
      std::vector<char> out(ml + e - s + 64 + (pad ? ml : 0));
      int64_t n = 0;
      int st = dna_fasta_interval(fa, chr.c_str(), s, e, ml, pad, 0, out.data(), (int64_t)out.size(), &n);
      CHECK(st == 0 && std::string(out.data(), n) == want, "fasta %s:%lld-%lld", chr.c_str(), s, e);
      ++nf;
    }
  }
  free(line);
  fclose(f);

  // single encodes (with a deliberately short output buffer on every third case)
  for (size_t i = 0; i < cases.size(); ++i) {
    const auto& c = cases[i];
    std::vector<int32_t> ids(c.win.size() + 8);
    int n = dna_bpe_encode(bpe, c.win.data(), (int)c.win.size(), ids.data(), (int)ids.size());
    // full ids carry [CLS] ... [SEP]
    CHECK(n + 2 == (int)c.full.size(), "bpe count case %zu", i);
    for (int k = 0; k < n && k + 1 < (int)c.full.size(); ++k) CHECK(ids[k] == c.full[k + 1], "bpe id case %zu", i);
    if (i % 3 == 0 && n > 2) {
      std::vector<int32_t> small(2);
      int n2 = dna_bpe_encode(bpe, c.win.data(), (int)c.win.size(), small.data(), 2);
      CHECK(n2 == n, "bpe short-buffer count case %zu", i);
    }
  }
  // batched dataset-form encode, 4 threads, then again in a forked child (DataLoader worker)
  auto batch_check = [&](const char* who) {
    const int P = cases.empty() ? 0 : cases[0].P;
    std::vector<const char*> seqs;
    std::vector<int> lens;
    for (const auto& c : cases) { seqs.push_back(c.win.data()); lens.push_back((int)c.win.size()); }
    const int W = P - 2;
    std::vector<int32_t> out((size_t)cases.size() * W), outl(cases.size());
    int st = dna_bpe_encode_batch(bpe, seqs.data(), lens.data(), (int)cases.size(), P, 0, out.data(),
                                  outl.data(), 4);
    CHECK(st == 0, "%s batch status", who);
    for (size_t i = 0; i < cases.size(); ++i)
      for (int k = 0; k < W; ++k) CHECK(out[i * W + k] == cases[i].ds[k], "%s batch case %zu pos %d", who, i, k);
  };
  batch_check("parent");
  pid_t pid = fork();
  if (pid == 0) {
    batch_check("child");
    _exit(fails ? 1 : 0);
  }
  int wst = 0;
  waitpid(pid, &wst, 0);
  CHECK(WIFEXITED(wst) && WEXITSTATUS(wst) == 0, "forked worker");

  // masking: Philox draws, every output position consistent with the rules
  std::vector<int64_t> seq(512), os(512), lab(512);
  std::vector<uint8_t> msk(512);
  const int64_t special[5] = {0, 1, 2, 3, 4};
  for (int i = 0; i < 512; ++i) seq[i] = i < 500 ? 5 + (i * 37) % 4000 : 3;
  for (uint64_t sid = 0; sid < 64; ++sid) {
    int st = dna_bert_mask(seq.data(), 512, 4096, special, 5, 4, 3, 0.15f, 0.1f, 0.1f, 2222, sid,
                           os.data(), msk.data(), lab.data());
    CHECK(st == 0, "mask status");
    for (int i = 0; i < 512; ++i) {
      CHECK(!(msk[i] && seq[i] == 3), "pad masked");
      CHECK(lab[i] == (msk[i] ? seq[i] : -100), "labels");
      CHECK(msk[i] || os[i] == seq[i], "unmasked changed");
    }
  }
  dna_fasta_close(fa);
  dna_bpe_destroy(bpe);
  printf("asan driver: %zu bpe cases, %d fasta cases, %d failures\n", cases.size(), nf, fails);
  return fails ? 1 : 0;
}
