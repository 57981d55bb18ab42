// Host data path: BERT masking (hg38_dataset.py:238-286) and mmap FASTA windows
// (FastaInterval, hg38_dataset.py:40-124; pyfaidx replaced by an mmap reader over the .fai).
#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

#include "dna_amd.h"

namespace dna {
void set_error(const char* fmt, ...);

// Philox4x32-10, identical to the device version in common.h
static inline void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
static inline float u24(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
}  // namespace dna

extern "C" int dna_bert_mask_from_draws(const int64_t* seq, int n, const float* u1, const float* u2,
                                        const int64_t* rand_tok, int mask_id, int pad_id,
                                        float mask_prob, float rand_prob, float unchanged_prob,
                                        int64_t* out_seq, uint8_t* out_mask, int64_t* out_labels) {
  if (!seq || !u1 || !u2 || !rand_tok || !out_seq || !out_mask || !out_labels || n < 0) {
    dna::set_error("dna_bert_mask_from_draws: bad args");
    return DNA_ERR_INVALID;
  }
  // thresholds computed as the reference does in Python doubles, compared in fp32
  const float keep_mask = (float)(1.0 - (double)rand_prob - (double)unchanged_prob);
  const float rnd_hi = (float)(1.0 - (double)unchanged_prob);
  for (int i = 0; i < n; ++i) {
    const bool m = seq[i] != pad_id && u1[i] < mask_prob;
    out_mask[i] = m;
    out_labels[i] = m ? seq[i] : -100;
    int64_t v = seq[i];
    if (m && u2[i] < keep_mask) v = mask_id;
    else if (m && u2[i] >= keep_mask && u2[i] < rnd_hi) v = rand_tok[i];
    out_seq[i] = v;
  }
  return DNA_OK;
}

extern "C" int dna_bert_mask(const int64_t* seq, int n, int vocab, const int64_t* special_ids,
                             int n_special, int mask_id, int pad_id, float mask_prob,
                             float rand_prob, float unchanged_prob, uint64_t seed,
                             uint64_t sample_id, int64_t* out_seq, uint8_t* out_mask,
                             int64_t* out_labels) {
  if (!seq || !out_seq || !out_mask || !out_labels || n < 0 || vocab <= n_special) {
    dna::set_error("dna_bert_mask: bad args");
    return DNA_ERR_INVALID;
  }
  std::vector<float> u1(n), u2(n);
  std::vector<int64_t> rt(n);
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int i = 0; i < n; ++i) {
    uint32_t c[4] = {(uint32_t)i, (uint32_t)sample_id, (uint32_t)(sample_id >> 32), 0xB3u};
    dna::philox(c, k0, k1);
    u1[i] = dna::u24(c[0]);
    u2[i] = dna::u24(c[1]);
    // uniform id in [0, vocab) rejecting special ids (re-draw, like the reference's while loop)
    uint32_t cand[2] = {c[2], c[3]};
    int64_t t = -1;
    for (uint32_t attempt = 0; t < 0; ++attempt) {
      for (int k = 0; k < 2 && t < 0; ++k) {
        int64_t x = (int64_t)(((uint64_t)cand[k] * (uint64_t)vocab) >> 32);
        bool sp = false;
        for (int s = 0; s < n_special; ++s) sp |= special_ids[s] == x;
        if (!sp) t = x;
      }
      uint32_t d[4] = {(uint32_t)i, (uint32_t)sample_id, (uint32_t)(sample_id >> 32), 0xC0u + attempt};
      dna::philox(d, k0, k1);
      cand[0] = d[0];
      cand[1] = d[1];
    }
    rt[i] = t;
  }
  return dna_bert_mask_from_draws(seq, n, u1.data(), u2.data(), rt.data(), mask_id, pad_id,
                                  mask_prob, rand_prob, unchanged_prob, out_seq, out_mask,
                                  out_labels);
}

// ----------------------------------------------------------------------------------- FASTA
struct FaiRec {
  std::string name;
  int64_t length, offset, linebases, linewidth;
};

struct dna_fasta {
  int fd = -1;
  const char* data = nullptr;
  size_t size = 0;
  std::vector<FaiRec> recs;
  std::unordered_map<std::string, size_t> by_name;
  ~dna_fasta() {
    if (data) munmap((void*)data, size);
    if (fd >= 0) close(fd);
  }
};

static bool parse_fai(dna_fasta* h, const std::string& path) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char name[4096];
  long long len, off, lb, lw;
  while (fscanf(f, "%4095s %lld %lld %lld %lld", name, &len, &off, &lb, &lw) == 5)
    h->recs.push_back({name, len, off, lb, lw});
  fclose(f);
  return !h->recs.empty();
}

// Build the index by scanning (samtools faidx semantics: uniform line length per record).
static bool build_index(dna_fasta* h) {
  const char* d = h->data;
  const size_t n = h->size;
  size_t i = 0;
  while (i < n) {
    if (d[i] != '>') { ++i; continue; }
    size_t e = i + 1;
    while (e < n && d[e] != '\n') ++e;
    std::string hdr(d + i + 1, d + e);
    if (!hdr.empty() && hdr.back() == '\r') hdr.pop_back();
    std::string nm = hdr.substr(0, hdr.find_first_of(" \t"));
    FaiRec r{nm, 0, (int64_t)(e + 1), 0, 0};
    size_t p = e + 1;
    bool first = true;
    while (p < n && d[p] != '>') {
      size_t le = p;
      while (le < n && d[le] != '\n') ++le;
      int64_t bases = (int64_t)(le - p);
      int64_t width = (int64_t)(le - p + (le < n ? 1 : 0));
      if (bases > 0 && d[le - 1] == '\r') --bases;
      if (first) { r.linebases = bases; r.linewidth = width; first = false; }
      r.length += bases;
      p = le + 1;
    }
    if (r.linebases == 0) r.linebases = r.linewidth = 1;
    h->recs.push_back(r);
    i = p;
  }
  return !h->recs.empty();
}

extern "C" dna_fasta* dna_fasta_open(const char* path) {
  if (!path) { dna::set_error("dna_fasta_open: null path"); return nullptr; }
  dna_fasta* h = new dna_fasta();
  h->fd = open(path, O_RDONLY);
  struct stat st;
  if (h->fd < 0 || fstat(h->fd, &st) != 0) {
    dna::set_error("dna_fasta_open: cannot open %s", path);
    delete h;
    return nullptr;
  }
  h->size = (size_t)st.st_size;
  if (h->size) {
    void* p = mmap(nullptr, h->size, PROT_READ, MAP_SHARED, h->fd, 0);
    if (p == MAP_FAILED) { dna::set_error("dna_fasta_open: mmap failed"); delete h; return nullptr; }
    h->data = (const char*)p;
  }
  if (!parse_fai(h, std::string(path) + ".fai") && !build_index(h)) {
    dna::set_error("dna_fasta_open: no records in %s", path);
    delete h;
    return nullptr;
  }
  for (size_t i = 0; i < h->recs.size(); ++i) h->by_name[h->recs[i].name] = i;
  return h;
}

extern "C" void dna_fasta_close(dna_fasta* h) { delete h; }
extern "C" int dna_fasta_num_records(const dna_fasta* h) { return h ? (int)h->recs.size() : 0; }
extern "C" const char* dna_fasta_record_name(const dna_fasta* h, int i) {
  return (h && i >= 0 && i < (int)h->recs.size()) ? h->recs[i].name.c_str() : nullptr;
}
extern "C" int64_t dna_fasta_record_length(const dna_fasta* h, const char* name) {
  if (!h || !name) return -1;
  auto it = h->by_name.find(name);
  return it == h->by_name.end() ? -1 : h->recs[it->second].length;
}

static inline char comp(char c) {
  switch (c) {
    case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A';
    case 'a': return 't'; case 'c': return 'g'; case 'g': return 'c'; case 't': return 'a';
    default: return c;
  }
}

extern "C" int dna_fasta_interval(const dna_fasta* h, const char* name, int64_t start, int64_t end,
                                  int64_t max_length, int pad_interval, int rc, char* out,
                                  int64_t cap, int64_t* out_len) {
  if (!h || !name || !out || !out_len) { dna::set_error("dna_fasta_interval: bad args"); return DNA_ERR_INVALID; }
  auto it = h->by_name.find(name);
  if (it == h->by_name.end()) { dna::set_error("dna_fasta_interval: no record %s", name); return DNA_ERR_INVALID; }
  const FaiRec& r = h->recs[it->second];
  const int64_t L = r.length;
  const int64_t interval = end - start;
  int64_t lpad = 0, rpad = 0;
  if (interval < max_length) {  // centre-expand (hg38_dataset.py:94-102)
    int64_t extra = max_length - interval;
    start -= extra / 2;
    end += extra - extra / 2;
  }
  if (start < 0) { lpad = -start; start = 0; }
  if (end > L) { rpad = end - L; end = L; }
  if (interval > max_length) end = start + max_length;  // keep the first max_length bp
  int64_t n = std::max<int64_t>(0, end - start);
  // pyfaidx slicing past the end returns what exists
  if (start > L) n = 0;
  const int64_t total = n + (pad_interval ? lpad + rpad : 0);
  if (total > cap) { dna::set_error("dna_fasta_interval: buffer too small (%lld)", (long long)total); return DNA_ERR_NOMEM; }
  // reference order: slice -> reverse-complement (rc_aug) -> '.' padding (hg38_dataset.py:116-122)
  char* core = out + (pad_interval ? lpad : 0);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t p = start + i;
    const int64_t off = r.offset + (p / r.linebases) * r.linewidth + p % r.linebases;
    core[i] = (off >= 0 && (size_t)off < h->size) ? h->data[off] : 'N';
  }
  if (rc) {
    std::reverse(core, core + n);
    for (int64_t i = 0; i < n; ++i) core[i] = comp(core[i]);
  }
  if (pad_interval) {
    memset(out, '.', lpad);
    memset(core + n, '.', rpad);
  }
  *out_len = total;
  return DNA_OK;
}
