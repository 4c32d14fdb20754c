// Native serving runtime: paged-KV block manager with prefix caching, plus the per-step
// batch-metadata builder.  (SURVEY §2.6 P4 / §7.1 `kv/block_manager.py`: the reference
// delegates continuous batching and KV paging to vLLM — llm/serve_llm.py:362-378 — so
// this is a new native component.)
//
// Design for the agent fan-out workload: N agent-b prompts share a long
// templated prefix, so full KV blocks are content-hashed (chained hash over the block's
// tokens and its predecessor's hash) and reused across sequences.  Freed blocks that
// carry a hash stay resident in an LRU "evictable" pool and are only recycled when the
// free list is empty, so consecutive workflow iterations hit the cache too.
//
// Everything here is O(blocks touched) per call and runs on the engine thread; Python
// calls it once per admitted sequence and once per step (build_batch).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <list>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t hash_block(uint64_t parent, const int64_t* toks, int n) {
  uint64_t h = mix64(parent ^ 0x51ED270B27D4A3F1ull);
  for (int i = 0; i < n; ++i) h = mix64(h ^ static_cast<uint64_t>(toks[i]) * 0x100000001B3ull);
  return h == 0 ? 1 : h;  // 0 means "no hash"
}

struct SeqState {
  std::vector<int32_t> blocks;
  std::vector<uint64_t> hashes;  // hashes of the leading full, committed blocks
};

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size, bool prefix_caching)
      : num_blocks_(num_blocks),
        block_size_(block_size),
        prefix_caching_(prefix_caching),
        ref_(num_blocks, 0),
        hash_(num_blocks, 0),
        lru_pos_(num_blocks) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad block manager size");
    free_.reserve(num_blocks);
    for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
    in_lru_.assign(num_blocks, false);
  }

  int num_free_blocks() const { return static_cast<int>(free_.size() + lru_.size()); }
  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int num_cached_blocks() const { return static_cast<int>(map_.size()); }
  int64_t prefix_queries() const { return queries_; }
  int64_t prefix_hits() const { return hits_; }

  int blocks_needed(int64_t num_tokens) const {
    return static_cast<int>((num_tokens + block_size_ - 1) / block_size_);
  }

  // Number of leading prompt tokens whose KV is already cached (multiple of block size,
  // always < prompt length so the last token is recomputed for its logits).
  int64_t peek_cached(py::array_t<int64_t, py::array::c_style> tokens) const {
    if (!prefix_caching_) return 0;
    auto buf = tokens.unchecked<1>();
    const int64_t n = buf.shape(0);
    const int64_t full = (n - 1) / block_size_;
    uint64_t h = 0;
    int64_t cached = 0;
    for (int64_t i = 0; i < full; ++i) {
      h = hash_block(h, buf.data(i * block_size_), block_size_);
      if (map_.find(h) == map_.end()) break;
      cached += block_size_;
    }
    return cached;
  }

  // Admit a new sequence.  Returns the number of prompt tokens served from the prefix
  // cache, or -1 if there are not enough blocks (nothing is changed in that case).
  int64_t allocate(int64_t seq_id, py::array_t<int64_t, py::array::c_style> tokens,
                   int64_t reserve_tokens) {
    if (seqs_.count(seq_id)) throw std::runtime_error("sequence already allocated");
    auto buf = tokens.unchecked<1>();
    const int64_t n = buf.shape(0);
    const int64_t want = std::max<int64_t>(n, reserve_tokens);
    const int total_blocks = blocks_needed(want);
    // -- prefix lookup
    std::vector<int32_t> hit_blocks;
    std::vector<uint64_t> hit_hashes;
    if (prefix_caching_) {
      const int64_t full = (n - 1) / block_size_;
      uint64_t h = 0;
      for (int64_t i = 0; i < full; ++i) {
        h = hash_block(h, buf.data(i * block_size_), block_size_);
        auto it = map_.find(h);
        if (it == map_.end()) break;
        hit_blocks.push_back(it->second);
        hit_hashes.push_back(h);
      }
    }
    // blocks from the evictable pool that we are about to revive do not count as free
    int revive = 0;
    for (int32_t b : hit_blocks)
      if (ref_[b] == 0) ++revive;
    const int fresh = total_blocks - static_cast<int>(hit_blocks.size());
    if (fresh > num_free_blocks() - revive) return -1;
    queries_ += (n - 1) / block_size_;
    hits_ += static_cast<int64_t>(hit_blocks.size());
    SeqState st;
    for (size_t i = 0; i < hit_blocks.size(); ++i) {
      take(hit_blocks[i]);
      st.blocks.push_back(hit_blocks[i]);
      st.hashes.push_back(hit_hashes[i]);
    }
    for (int i = 0; i < fresh; ++i) st.blocks.push_back(pop_free());
    seqs_.emplace(seq_id, std::move(st));
    return static_cast<int64_t>(hit_blocks.size()) * block_size_;
  }

  // Make sure `seq_id` owns enough blocks for `num_tokens` tokens.  Returns false (and
  // changes nothing) when the pool is exhausted.
  bool ensure(int64_t seq_id, int64_t num_tokens) {
    auto& st = get(seq_id);
    const int need = blocks_needed(num_tokens) - static_cast<int>(st.blocks.size());
    if (need <= 0) return true;
    if (need > num_free_blocks()) return false;
    for (int i = 0; i < need; ++i) st.blocks.push_back(pop_free());
    return true;
  }

  // Register content hashes for blocks that became full now that `num_computed` tokens
  // of `tokens` have their KV written.
  void commit(int64_t seq_id, py::array_t<int64_t, py::array::c_style> tokens,
              int64_t num_computed) {
    if (!prefix_caching_) return;
    auto& st = get(seq_id);
    auto buf = tokens.unchecked<1>();
    const int64_t full = std::min<int64_t>(num_computed, buf.shape(0)) / block_size_;
    uint64_t h = st.hashes.empty() ? 0 : st.hashes.back();
    for (int64_t i = static_cast<int64_t>(st.hashes.size()); i < full; ++i) {
      if (i >= static_cast<int64_t>(st.blocks.size())) break;
      h = hash_block(h, buf.data(i * block_size_), block_size_);
      st.hashes.push_back(h);
      const int32_t b = st.blocks[i];
      if (hash_[b] == 0 && map_.find(h) == map_.end()) {
        hash_[b] = h;
        map_.emplace(h, b);
      }
    }
  }

  void free(int64_t seq_id) {
    auto it = seqs_.find(seq_id);
    if (it == seqs_.end()) return;
    // release in reverse so the tail of a sequence is evicted before its shared prefix
    for (auto b = it->second.blocks.rbegin(); b != it->second.blocks.rend(); ++b) release(*b);
    seqs_.erase(it);
  }

  std::vector<int32_t> blocks(int64_t seq_id) { return get(seq_id).blocks; }
  bool has(int64_t seq_id) const { return seqs_.count(seq_id) != 0; }

  void reset_prefix_cache() {
    for (int32_t b : lru_) {
      in_lru_[b] = false;
      map_.erase(hash_[b]);
      hash_[b] = 0;
      free_.push_back(b);
    }
    lru_.clear();
  }

  // ---- per-step metadata ---------------------------------------------------------------
  // seq_ids[S], q_start[S] (= tokens already in cache), q_len[S].  Returns a dict of numpy
  // arrays: positions/slot_mapping (int32 [T']), block_tables (int32 [S', width]),
  // seq_kvlen (int32 [S']), seq_qstart (int32 [S'+1]), logits_idx (int64 [S']), and the
  // prefill tiling tile_seq/tile_qoff (int32; `tile_tokens` query tokens per tile, only for
  // sequences with index >= tile_from).
  // Padding (hipGraph buckets): sequences S..pad_seqs-1 are dummies with one query row
  // each, kvlen 0 and slot -1 (kernels skip them); rows past that up to pad_tokens get
  // slot -1 and belong to no sequence.
  py::dict build_batch(py::array_t<int64_t, py::array::c_style> seq_ids,
                       py::array_t<int64_t, py::array::c_style> q_start,
                       py::array_t<int64_t, py::array::c_style> q_len, int bt_width,
                       int tile_tokens, int tile_from, int pad_tokens, int pad_seqs) {
    auto ids = seq_ids.unchecked<1>();
    auto qs = q_start.unchecked<1>();
    auto ql = q_len.unchecked<1>();
    const int64_t S = ids.shape(0);
    int64_t T = 0;
    for (int64_t i = 0; i < S; ++i) T += ql(i);
    const int64_t Sp = std::max<int64_t>(S, pad_seqs);
    const int64_t Tp = std::max<int64_t>(T + (Sp - S), pad_tokens);
    py::array_t<int32_t> positions(Tp), slots(Tp);
    py::array_t<int64_t> logits_idx(Sp);
    py::array_t<int32_t> bt({Sp, static_cast<int64_t>(bt_width)});
    py::array_t<int32_t> kvlen(Sp), qstart(Sp + 1);
    auto P = positions.mutable_unchecked<1>();
    auto SL = slots.mutable_unchecked<1>();
    auto LI = logits_idx.mutable_unchecked<1>();
    auto BT = bt.mutable_unchecked<2>();
    auto KV = kvlen.mutable_unchecked<1>();
    auto QS = qstart.mutable_unchecked<1>();
    std::vector<int32_t> tseq, toff;
    int64_t row = 0;
    for (int64_t i = 0; i < S; ++i) {
      const auto& st = get(ids(i));
      const int64_t start = qs(i), len = ql(i);
      const int need = blocks_needed(start + len);
      if (static_cast<int64_t>(st.blocks.size()) < need)
        throw std::runtime_error("build_batch: sequence has too few blocks");
      if (need > bt_width) throw std::runtime_error("build_batch: block table width too small");
      QS(i) = static_cast<int32_t>(row);
      KV(i) = static_cast<int32_t>(start + len);
      for (int64_t j = 0; j < len; ++j) {
        const int64_t pos = start + j;
        P(row + j) = static_cast<int32_t>(pos);
        SL(row + j) = static_cast<int32_t>(st.blocks[pos / block_size_] * block_size_ +
                                           pos % block_size_);
      }
      const int nb = std::min<int>(bt_width, static_cast<int>(st.blocks.size()));
      for (int b = 0; b < nb; ++b) BT(i, b) = st.blocks[b];
      for (int b = nb; b < bt_width; ++b) BT(i, b) = 0;
      if (tile_tokens > 0 && i >= tile_from)
        for (int64_t o = 0; o < len; o += tile_tokens) {
          tseq.push_back(static_cast<int32_t>(i));
          toff.push_back(static_cast<int32_t>(o));
        }
      row += len;
      LI(i) = row - 1;
    }
    for (int64_t i = S; i < Sp; ++i) {
      QS(i) = static_cast<int32_t>(row);
      KV(i) = 0;
      P(row) = 0;
      SL(row) = -1;
      for (int b = 0; b < bt_width; ++b) BT(i, b) = 0;
      ++row;
      LI(i) = row - 1;
    }
    QS(Sp) = static_cast<int32_t>(row);
    for (int64_t j = row; j < Tp; ++j) {
      P(j) = 0;
      SL(j) = -1;
    }
    py::array_t<int32_t> ts(static_cast<int64_t>(tseq.size())), to(static_cast<int64_t>(toff.size()));
    if (!tseq.empty()) {
      std::copy(tseq.begin(), tseq.end(), ts.mutable_data());
      std::copy(toff.begin(), toff.end(), to.mutable_data());
    }
    py::dict d;
    d["positions"] = positions;
    d["slot_mapping"] = slots;
    d["block_tables"] = bt;
    d["seq_kvlen"] = kvlen;
    d["seq_qstart"] = qstart;
    d["tile_seq"] = ts;
    d["tile_qoff"] = to;
    d["logits_idx"] = logits_idx;
    d["num_tokens"] = T;
    return d;
  }

 private:
  SeqState& get(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) throw std::runtime_error("unknown sequence id");
    return it->second;
  }
  const SeqState& get(int64_t id) const {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) throw std::runtime_error("unknown sequence id");
    return it->second;
  }

  void take(int32_t b) {
    if (ref_[b] == 0 && in_lru_[b]) {
      lru_.erase(lru_pos_[b]);
      in_lru_[b] = false;
    }
    ++ref_[b];
  }

  int32_t pop_free() {
    int32_t b;
    if (!free_.empty()) {
      b = free_.back();
      free_.pop_back();
    } else {
      if (lru_.empty()) throw std::runtime_error("KV block pool exhausted");
      b = lru_.front();  // least recently released cached block
      lru_.pop_front();
      in_lru_[b] = false;
      map_.erase(hash_[b]);
      hash_[b] = 0;
    }
    ref_[b] = 1;
    return b;
  }

  void release(int32_t b) {
    if (--ref_[b] > 0) return;
    if (hash_[b] != 0) {
      lru_.push_back(b);
      lru_pos_[b] = std::prev(lru_.end());
      in_lru_[b] = true;
    } else {
      free_.push_back(b);
    }
  }

  int num_blocks_;
  int block_size_;
  bool prefix_caching_;
  std::vector<int32_t> ref_;
  std::vector<uint64_t> hash_;
  std::vector<std::list<int32_t>::iterator> lru_pos_;
  std::vector<bool> in_lru_;
  std::vector<int32_t> free_;
  std::list<int32_t> lru_;
  std::unordered_map<uint64_t, int32_t> map_;
  std::unordered_map<int64_t, SeqState> seqs_;
  int64_t queries_ = 0;
  int64_t hits_ = 0;
};

}  // namespace

void register_block_manager(py::module_& m) {
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int, bool>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("prefix_caching") = true)
      .def("num_free_blocks", &BlockManager::num_free_blocks)
      .def("num_blocks", &BlockManager::num_blocks)
      .def("block_size", &BlockManager::block_size)
      .def("num_cached_blocks", &BlockManager::num_cached_blocks)
      .def("prefix_queries", &BlockManager::prefix_queries)
      .def("prefix_hits", &BlockManager::prefix_hits)
      .def("blocks_needed", &BlockManager::blocks_needed)
      .def("peek_cached", &BlockManager::peek_cached)
      .def("allocate", &BlockManager::allocate, py::arg("seq_id"), py::arg("tokens"),
           py::arg("reserve_tokens") = 0)
      .def("ensure", &BlockManager::ensure)
      .def("commit", &BlockManager::commit)
      .def("free", &BlockManager::free)
      .def("blocks", &BlockManager::blocks)
      .def("has", &BlockManager::has)
      .def("reset_prefix_cache", &BlockManager::reset_prefix_cache)
      .def("build_batch", &BlockManager::build_batch, py::arg("seq_ids"), py::arg("q_start"),
           py::arg("q_len"), py::arg("bt_width"), py::arg("tile_tokens") = 0,
           py::arg("tile_from") = 0, py::arg("pad_tokens") = 0, py::arg("pad_seqs") = 0);
}
