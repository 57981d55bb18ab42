// Byte-pair-encoding tokenizer for the DNABERT-2 vocabulary (host C++, C ABI).
//
// Bit-exact restatement of the HF `tokenizers` BPE model (Rust; pinned 0.13.3 by the reference,
// /root/reference/requirements.txt:106) for DNABERT-2-117M/tokenizer.json: added-token split,
// `Whitespace` pre-tokenizer (\w+|[^\w\s]+), per-character symbols with [UNK] for unknown
// characters (fuse_unk = false), then merges from a min-heap ordered by (merge rank, position),
// re-validating each popped entry against the current pair (tokenizers models/bpe/word.rs).
// Called per sample at src/dataloaders/datasets/hg38_dataset.py:369-379 in the reference.
// The handle is immutable after creation: safe across threads and fork()ed DataLoader workers.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "dna_amd.h"

namespace dna {
void set_error(const char* fmt, ...);

// ------------------------------------------------------------------------------- minimal JSON
struct JVal {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  double num = 0;
  bool b = false;
  std::string s;
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;
  const JVal* get(const char* k) const {
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

class JParser {
 public:
  explicit JParser(const std::string& t) : t_(t) {}
  bool parse(JVal& v) {
    ws();
    if (!value(v)) return false;
    ws();
    return p_ == t_.size();
  }

 private:
  const std::string& t_;
  size_t p_ = 0;
  void ws() {
    while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\n' || t_[p_] == '\r' || t_[p_] == '\t')) ++p_;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
    } else {
      o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
      o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
    }
  }
  bool hex4(uint32_t& cp) {
    if (p_ + 4 > t_.size()) return false;
    cp = 0;
    for (int i = 0; i < 4; ++i) {
      char c = t_[p_++];
      cp <<= 4;
      if (c >= '0' && c <= '9') cp |= c - '0';
      else if (c >= 'a' && c <= 'f') cp |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') cp |= c - 'A' + 10;
      else return false;
    }
    return true;
  }
  bool str(std::string& o) {
    if (t_[p_] != '"') return false;
    ++p_;
    while (p_ < t_.size() && t_[p_] != '"') {
      char c = t_[p_++];
      if (c != '\\') { o += c; continue; }
      if (p_ >= t_.size()) return false;
      char e = t_[p_++];
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp;
          if (!hex4(cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00 && p_ + 6 <= t_.size() && t_[p_] == '\\' && t_[p_ + 1] == 'u') {
            p_ += 2;
            uint32_t lo;
            if (!hex4(lo)) return false;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(o, cp);
          break;
        }
        default: return false;
      }
    }
    if (p_ >= t_.size()) return false;
    ++p_;
    return true;
  }
  bool value(JVal& v) {
    if (p_ >= t_.size()) return false;
    char c = t_[p_];
    if (c == '{') {
      v.kind = JVal::OBJ;
      ++p_;
      ws();
      if (p_ < t_.size() && t_[p_] == '}') { ++p_; return true; }
      while (true) {
        ws();
        std::string k;
        if (!str(k)) return false;
        ws();
        if (p_ >= t_.size() || t_[p_] != ':') return false;
        ++p_;
        ws();
        v.obj.emplace_back(std::move(k), JVal());
        if (!value(v.obj.back().second)) return false;
        ws();
        if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
        if (p_ < t_.size() && t_[p_] == '}') { ++p_; return true; }
        return false;
      }
    }
    if (c == '[') {
      v.kind = JVal::ARR;
      ++p_;
      ws();
      if (p_ < t_.size() && t_[p_] == ']') { ++p_; return true; }
      while (true) {
        ws();
        v.arr.emplace_back();
        if (!value(v.arr.back())) return false;
        ws();
        if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
        if (p_ < t_.size() && t_[p_] == ']') { ++p_; return true; }
        return false;
      }
    }
    if (c == '"') { v.kind = JVal::STR; return str(v.s); }
    if (t_.compare(p_, 4, "true") == 0) { v.kind = JVal::BOOL; v.b = true; p_ += 4; return true; }
    if (t_.compare(p_, 5, "false") == 0) { v.kind = JVal::BOOL; p_ += 5; return true; }
    if (t_.compare(p_, 4, "null") == 0) { v.kind = JVal::NUL; p_ += 4; return true; }
    size_t st = p_;
    while (p_ < t_.size() && (isdigit((unsigned char)t_[p_]) || strchr("+-.eE", t_[p_]))) ++p_;
    if (st == p_) return false;
    v.kind = JVal::NUM;
    v.num = strtod(t_.substr(st, p_ - st).c_str(), nullptr);
    return true;
  }
};

// ------------------------------------------------------------------------------- merge table
// open addressing on (left id, right id) -> (rank, new id)
class MergeTable {
 public:
  void init(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    keys_.assign(cap, ~0ull);
    vals_.assign(cap, {0, 0});
    mask_ = cap - 1;
  }
  void put(int a, int b, int rank, int nid) {
    uint64_t k = key(a, b);
    size_t i = hash(k) & mask_;
    while (keys_[i] != ~0ull && keys_[i] != k) i = (i + 1) & mask_;
    if (keys_[i] == ~0ull) { keys_[i] = k; vals_[i] = {rank, nid}; }
  }
  // returns false when (a, b) is not a merge
  inline bool get(int a, int b, int& rank, int& nid) const {
    uint64_t k = key(a, b);
    size_t i = hash(k) & mask_;
    while (true) {
      uint64_t kk = keys_[i];
      if (kk == k) { rank = vals_[i].first; nid = vals_[i].second; return true; }
      if (kk == ~0ull) return false;
      i = (i + 1) & mask_;
    }
  }

 private:
  static uint64_t key(int a, int b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }
  static size_t hash(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return (size_t)k;
  }
  std::vector<uint64_t> keys_;
  std::vector<std::pair<int, int>> vals_;
  size_t mask_ = 0;
};

}  // namespace dna

struct dna_bpe {
  std::unordered_map<std::string, int> vocab;
  int byte_id[256];
  dna::MergeTable merges;
  std::vector<std::pair<std::string, int>> added;  // longest first
  int unk = 0, cls = 1, sep = 2, pad = 3;
  int vocab_size = 0;
};

namespace {

struct HeapEnt {
  int rank, pos, nid;
  // std heap is a max-heap: "less" means lower priority = higher rank, then higher pos
  bool operator<(const HeapEnt& o) const { return rank != o.rank ? rank > o.rank : pos > o.pos; }
};

struct Scratch {
  std::vector<int> id, prev, next;
  std::vector<unsigned char> alive;
  std::vector<HeapEnt> heap;
};

inline bool is_space(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
// \w for ASCII; bytes >= 0x80 (UTF-8 sequences) are treated as word characters.
inline bool is_word(unsigned char c) { return isalnum(c) || c == '_' || c >= 0x80; }

void bpe_word(const dna_bpe& h, const char* w, int n, Scratch& sc, std::vector<int32_t>& out) {
  sc.id.clear();
  for (int i = 0; i < n;) {
    unsigned char c = (unsigned char)w[i];
    if (c < 0x80) {
      int id = h.byte_id[c];
      sc.id.push_back(id >= 0 ? id : h.unk);
      ++i;
    } else {  // one UTF-8 character
      int len = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 1;
      len = std::min(len, n - i);
      auto it = h.vocab.find(std::string(w + i, len));
      sc.id.push_back(it != h.vocab.end() ? it->second : h.unk);
      i += len;
    }
  }
  const int m = (int)sc.id.size();
  sc.prev.resize(m);
  sc.next.resize(m);
  sc.alive.assign(m, 1);
  for (int i = 0; i < m; ++i) { sc.prev[i] = i - 1; sc.next[i] = i + 1 < m ? i + 1 : -1; }
  auto& heap = sc.heap;
  heap.clear();
  for (int i = 0; i + 1 < m; ++i) {
    int r, nid;
    if (h.merges.get(sc.id[i], sc.id[i + 1], r, nid)) heap.push_back({r, i, nid});
  }
  std::make_heap(heap.begin(), heap.end());
  while (!heap.empty()) {
    std::pop_heap(heap.begin(), heap.end());
    HeapEnt top = heap.back();
    heap.pop_back();
    const int pos = top.pos;
    if (!sc.alive[pos] || sc.next[pos] < 0) continue;
    const int r = sc.next[pos];
    int cr, cnid;
    if (!h.merges.get(sc.id[pos], sc.id[r], cr, cnid) || cnid != top.nid) continue;
    sc.id[pos] = top.nid;
    sc.alive[r] = 0;
    sc.next[pos] = sc.next[r];
    if (sc.next[r] >= 0) sc.prev[sc.next[r]] = pos;
    int rk, nid;
    const int pv = sc.prev[pos];
    if (pv >= 0 && h.merges.get(sc.id[pv], sc.id[pos], rk, nid)) {
      heap.push_back({rk, pv, nid});
      std::push_heap(heap.begin(), heap.end());
    }
    const int nx = sc.next[pos];
    if (nx >= 0 && h.merges.get(sc.id[pos], sc.id[nx], rk, nid)) {
      heap.push_back({rk, pos, nid});
      std::push_heap(heap.begin(), heap.end());
    }
  }
  for (int i = 0; i < m; ++i)
    if (sc.alive[i]) out.push_back(sc.id[i]);
}

void pretok_and_bpe(const dna_bpe& h, const char* t, int n, Scratch& sc, std::vector<int32_t>& out) {
  int i = 0;
  while (i < n) {
    unsigned char c = (unsigned char)t[i];
    if (is_space(c)) { ++i; continue; }
    const bool wcls = is_word(c);
    int j = i + 1;
    while (j < n) {
      unsigned char d = (unsigned char)t[j];
      if (is_space(d) || is_word(d) != wcls) break;
      ++j;
    }
    bpe_word(h, t + i, j - i, sc, out);
    i = j;
  }
}

void encode(const dna_bpe& h, const char* t, int n, Scratch& sc, std::vector<int32_t>& out) {
  out.clear();
  int seg = 0;
  for (int i = 0; i < n;) {
    int hit = -1;
    if (t[i] == '[') {
      for (size_t a = 0; a < h.added.size(); ++a) {
        const std::string& s = h.added[a].first;
        if ((int)s.size() <= n - i && memcmp(t + i, s.data(), s.size()) == 0) { hit = (int)a; break; }
      }
    }
    if (hit < 0) { ++i; continue; }
    pretok_and_bpe(h, t + seg, i - seg, sc, out);
    out.push_back(h.added[hit].second);
    i += (int)h.added[hit].first.size();
    seg = i;
  }
  pretok_and_bpe(h, t + seg, n - seg, sc, out);
}

}  // namespace

extern "C" dna_bpe* dna_bpe_create(const char* json_path) {
  if (!json_path) { dna::set_error("dna_bpe_create: null path"); return nullptr; }
  std::ifstream f(json_path, std::ios::binary);
  if (!f) { dna::set_error("dna_bpe_create: cannot open %s", json_path); return nullptr; }
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  dna::JVal root;
  if (!dna::JParser(text).parse(root) || root.kind != dna::JVal::OBJ) {
    dna::set_error("dna_bpe_create: malformed JSON in %s", json_path);
    return nullptr;
  }
  std::unique_ptr<dna_bpe> h(new dna_bpe());
  std::vector<std::pair<std::string, std::string>> merges;
  std::string unk = "[UNK]";
  const dna::JVal* fmt = root.get("format");
  try {
    if (fmt && fmt->s == "dna_amd-bpe-v1") {
      const dna::JVal* toks = root.get("tokens");
      for (size_t i = 0; i < toks->arr.size(); ++i) h->vocab[toks->arr[i].s] = (int)i;
      for (auto& m : root.get("merges")->arr) merges.emplace_back(m.arr.at(0).s, m.arr.at(1).s);
      for (auto& kv : root.get("special_tokens")->obj) h->added.emplace_back(kv.first, (int)kv.second.num);
      unk = root.get("unk_token")->s;
    } else {
      const dna::JVal* model = root.get("model");
      if (!model || !model->get("vocab") || !model->get("merges")) throw std::runtime_error("no model");
      const dna::JVal* ty = model->get("type");
      if (ty && ty->s != "BPE") throw std::runtime_error("not a BPE model");
      for (auto& kv : model->get("vocab")->obj) h->vocab[kv.first] = (int)kv.second.num;
      for (auto& m : model->get("merges")->arr) {
        if (m.kind == dna::JVal::STR) {
          size_t sp = m.s.find(' ');
          if (sp == std::string::npos) throw std::runtime_error("bad merge");
          merges.emplace_back(m.s.substr(0, sp), m.s.substr(sp + 1));
        } else {
          merges.emplace_back(m.arr.at(0).s, m.arr.at(1).s);
        }
      }
      if (const dna::JVal* at = root.get("added_tokens"))
        for (auto& a : at->arr) h->added.emplace_back(a.get("content")->s, (int)a.get("id")->num);
      if (const dna::JVal* u = model->get("unk_token")) unk = u->s;
    }
  } catch (const std::exception& e) {
    dna::set_error("dna_bpe_create: unexpected tokenizer layout (%s)", e.what());
    return nullptr;
  }
  auto need = [&](const std::string& k) -> int {
    auto it = h->vocab.find(k);
    if (it != h->vocab.end()) return it->second;
    for (auto& a : h->added) if (a.first == k) return a.second;
    return -1;
  };
  h->unk = need(unk);
  h->cls = need("[CLS]");
  h->sep = need("[SEP]");
  h->pad = need("[PAD]");
  if (h->unk < 0 || h->cls < 0 || h->sep < 0 || h->pad < 0) {
    dna::set_error("dna_bpe_create: special tokens missing");
    return nullptr;
  }
  for (int c = 0; c < 256; ++c) {
    auto it = c < 0x80 ? h->vocab.find(std::string(1, (char)c)) : h->vocab.end();
    h->byte_id[c] = it != h->vocab.end() ? it->second : -1;
  }
  h->merges.init(merges.size());
  for (size_t r = 0; r < merges.size(); ++r) {
    auto a = h->vocab.find(merges[r].first), b = h->vocab.find(merges[r].second);
    auto ab = h->vocab.find(merges[r].first + merges[r].second);
    if (a == h->vocab.end() || b == h->vocab.end() || ab == h->vocab.end()) {
      dna::set_error("dna_bpe_create: merge %zu refers to unknown tokens", r);
      return nullptr;
    }
    h->merges.put(a->second, b->second, (int)r, ab->second);
  }
  std::sort(h->added.begin(), h->added.end(),
            [](const std::pair<std::string, int>& x, const std::pair<std::string, int>& y) {
              return x.first.size() > y.first.size();
            });
  int mx = 0;
  for (auto& kv : h->vocab) mx = std::max(mx, kv.second + 1);
  for (auto& a : h->added) mx = std::max(mx, a.second + 1);
  h->vocab_size = mx;
  return h.release();
}

extern "C" void dna_bpe_destroy(dna_bpe* h) { delete h; }

extern "C" int dna_bpe_vocab_size(const dna_bpe* h) { return h ? h->vocab_size : -DNA_ERR_INVALID; }

extern "C" int dna_bpe_encode(const dna_bpe* h, const char* text, int len, int32_t* out_ids, int cap) {
  if (!h || (!text && len > 0) || len < 0) { dna::set_error("dna_bpe_encode: bad args"); return -DNA_ERR_INVALID; }
  Scratch sc;
  std::vector<int32_t> ids;
  encode(*h, text, len, sc, ids);
  const size_t n = std::min<size_t>(ids.size(), (size_t)std::max(cap, 0));
  if (out_ids && n > 0) memcpy(out_ids, ids.data(), sizeof(int32_t) * n);  // memcpy(.., null, 0) is UB
  return (int)ids.size();
}

extern "C" int dna_bpe_encode_batch(const dna_bpe* h, const char* const* seqs, const int* lens, int n,
                                    int pad_max_length, int add_eos, int32_t* out_ids,
                                    int32_t* out_lens, int nthreads) {
  if (!h || !seqs || !lens || !out_ids || n < 0 || pad_max_length < 2) {
    dna::set_error("dna_bpe_encode_batch: bad args");
    return DNA_ERR_INVALID;
  }
  const int P = pad_max_length, W = P - 2 + (add_eos ? 1 : 0);
  auto work = [&](int lo, int hi) {
    Scratch sc;
    std::vector<int32_t> ids;
    std::vector<int32_t> full(P);
    for (int i = lo; i < hi; ++i) {
      encode(*h, seqs[i], lens[i], sc, ids);
      const int body = std::min((int)ids.size(), P - 2);
      int k = 0;
      full[k++] = h->cls;
      for (int j = 0; j < body; ++j) full[k++] = ids[j];
      full[k++] = h->sep;
      while (k < P) full[k++] = h->pad;
      memcpy(out_ids + (size_t)i * W, full.data() + 1, sizeof(int32_t) * W);  // [1:-1] or [1:]
      if (out_lens) out_lens[i] = body;
    }
  };
  int nt = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = std::max(1, std::min(nt, n));
  if (nt == 1) {
    work(0, n);
  } else {
    std::vector<std::thread> th;
    const int chunk = (n + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
      int lo = t * chunk, hi = std::min(n, lo + chunk);
      if (lo < hi) th.emplace_back(work, lo, hi);
    }
    for (auto& x : th) x.join();
  }
  return DNA_OK;
}
