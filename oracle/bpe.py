"""Pure-Python restatement of the DNABERT-2 BPE tokenizer (TEST INFRASTRUCTURE).

Oracle only (tests/, smoke(), bench cpu_baseline). The reference tokenises with HF `tokenizers`
(Rust, pinned 0.13.3 in /root/reference/requirements.txt:106; not vendored) driven by
/root/reference/DNABERT-2-117M/tokenizer.json, called at hg38_dataset.py:369-379 with
padding="max_length", max_length=pad_max_length, truncation=True, then `[1:-1]`.
Published algorithm restated here (tokenizers `models/bpe/word.rs::merge_all`):
  * added/special tokens are split out of the raw text first;
  * `Whitespace` pre-tokenizer: words are matches of  \\w+|[^\\w\\s]+ ;
  * each word starts as one symbol per character (unknown char -> [UNK], fuse_unk = false);
  * a heap of candidate merges ordered by (merge rank, position) -- lowest rank first, leftmost on
    ties; a popped entry is applied only if its left symbol is alive, has a right neighbour, and
    the CURRENT pair maps to the entry's new id; after a merge the pairs with the previous and
    the next symbol are pushed.
Pinned bit-exact by tests/golden/tok_golden.npz (reference tokenizer run in this container).
"""
import heapq
import json
import re

_WORD = re.compile(r"\w+|[^\w\s]+")


class BPERef:
    def __init__(self, tokenizer_json: str):
        """Accepts an HF tokenizer.json or the repo's compact dna_amd/data/dnabert2_bpe.json."""
        t = json.load(open(tokenizer_json))
        if t.get("format") == "dna_amd-bpe-v1":
            self.vocab = {tok: i for i, tok in enumerate(t["tokens"])}
            merges, unk = t["merges"], t["unk_token"]
            self.added = dict(t["special_tokens"])
        else:
            m = t["model"]
            self.vocab = dict(m["vocab"])
            merges, unk = m["merges"], m["unk_token"]
            self.added = {a["content"]: a["id"] for a in t["added_tokens"]}
        self.unk_id = self.vocab[unk]
        self.merges = {}
        for rank, mg in enumerate(merges):
            a, b = mg.split(" ") if isinstance(mg, str) else mg
            self.merges[(self.vocab[a], self.vocab[b])] = (rank, self.vocab[a + b])
        self.cls_id, self.sep_id = self.added["[CLS]"], self.added["[SEP]"]
        self.pad_id, self.mask_id = self.added["[PAD]"], self.added["[MASK]"]

    # -- pre-tokenization ---------------------------------------------------------------
    def _split_added(self, text):
        if not any(a in text for a in self.added):
            return [(text, False)]
        pat = re.compile("|".join(re.escape(a) for a in sorted(self.added, key=len, reverse=True)))
        out, pos = [], 0
        for mt in pat.finditer(text):
            if mt.start() > pos:
                out.append((text[pos:mt.start()], False))
            out.append((mt.group(0), True))
            pos = mt.end()
        if pos < len(text):
            out.append((text[pos:], False))
        return out

    # -- BPE on one word ------------------------------------------------------------------
    def bpe_word(self, word):
        ids = [self.vocab.get(ch, self.unk_id) for ch in word]
        n = len(ids)
        prev = list(range(-1, n - 1))
        nxt = list(range(1, n + 1))
        nxt[-1] = -1 if n else -1
        alive = [True] * n
        heap = []
        for i in range(n - 1):
            mg = self.merges.get((ids[i], ids[i + 1]))
            if mg:
                heap.append((mg[0], i, mg[1]))
        heapq.heapify(heap)
        while heap:
            rank, pos, new_id = heapq.heappop(heap)
            if not alive[pos] or nxt[pos] == -1:
                continue
            r = nxt[pos]
            cur = self.merges.get((ids[pos], ids[r]))
            if cur is None or cur[1] != new_id:
                continue
            ids[pos] = new_id
            alive[r] = False
            nxt[pos] = nxt[r]
            if nxt[r] != -1:
                prev[nxt[r]] = pos
            if prev[pos] != -1:
                mg = self.merges.get((ids[prev[pos]], ids[pos]))
                if mg:
                    heapq.heappush(heap, (mg[0], prev[pos], mg[1]))
            if nxt[pos] != -1:
                mg = self.merges.get((ids[pos], ids[nxt[pos]]))
                if mg:
                    heapq.heappush(heap, (mg[0], pos, mg[1]))
        return [ids[i] for i in range(n) if alive[i]]

    def encode(self, text, add_special_tokens=False):
        out = []
        for piece, is_added in self._split_added(text):
            if is_added:
                out.append(self.added[piece])
                continue
            for w in _WORD.findall(piece):
                out.extend(self.bpe_word(w))
        if add_special_tokens:
            out = [self.cls_id] + out + [self.sep_id]
        return out

    def encode_dataset(self, text, pad_max_length, add_eos=False):
        """hg38_dataset.py:369-379: pad to max_length P with truncation, then drop CLS (and the
        last element unless add_eos)."""
        body = self.encode(text)[: pad_max_length - 2]
        ids = [self.cls_id] + body + [self.sep_id]
        ids += [self.pad_id] * (pad_max_length - len(ids))
        return ids[1:] if add_eos else ids[1:-1]
