// engine.h -- symbolic GF(2^8) row algebra and device-program builder.
//
// The control plane (encoder.cpp / decoder.cpp) restates the reference state machines exactly,
// but every byte buffer of the reference (original packets, running sums, recovery packets,
// the product workspace, the decoder's recovery rows) is replaced by a symbolic value:
//
//     value = XOR over terms of  coef * row[0:len]      (rows zero-padded beyond their data)
//
// where `row` is a row of the device arena (HBM).  Every reference gf256_add_mem /
// gf256_muladd_mem / gf256_mul_mem call becomes a term-list operation on the host, and the
// values are only *materialized* (an op in the device program) when a result must exist in
// memory: a recovery packet, a recovered original, a running-sum snapshot, or a decoder
// elimination ("partial") row.  Because GF(2^8) arithmetic is exact, associative and
// commutative, the device reproduces the reference bytes exactly no matter how the terms are
// grouped or ordered.
//
// Running sums (SiameseEncoder.cpp:359-418, SiameseDecoder.cpp:1538-1739) are Chains: an
// in-order list of accumulated terms with snapshot points, executed on the device as ONE scan
// op per chain per flush (one wave walks the chain for its byte slice and stores a snapshot row
// at each point), so long sums cost one read per accumulated row, not one per recovery.
//
// Levels: a row written by an op in the pending program has level >= 1; ops run level by level
// (one launch per level), so an op only reads rows of lower levels.  Materialization policies
// keep the level count small and independent of the number of solves in a flush.
#pragma once

#include "program.h"
#include "gf256.h"

#include <stdint.h>
#include <vector>
#include <algorithm>
#include <memory>
#include <utility>

namespace tamd {

using RowId = uint32_t;  // handle into RowTable (not an arena offset)
static const RowId kNoRow = 0xffffffffu;

struct Term {
    RowId row;
    uint32_t len;
    uint8_t coef;
};
// A term whose row has this bit set names a run of level-0 rows registered with the pending
// program (ProgramBuilder::run_term) instead of one row: coef * sum_k c_k * row_k[0:len].
static const RowId kRunFlag = 0x80000000u;
inline bool is_run(RowId r) { return (r & kRunFlag) != 0; }

// Allocator whose value-initialisation leaves PODs uninitialised: growing a term list or an
// instruction list by resize() and then writing every new element skips a zero fill.
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind { typedef NoInitAlloc<U> other; };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept { ::new ((void*)p) U; }
    template <class U, class... A>
    void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};

// A symbolic buffer.  `terms` may contain duplicates; they are merged when materialized.
typedef std::vector<Term, NoInitAlloc<Term>> Sym;
typedef std::vector<tamd_instr, NoInitAlloc<tamd_instr>> InstrVec;

// Bytes of an op one device work item covers (program.h): TAMD_SLICE_BYTES_X (tamd_exec24) unless
// TONK_AMD_SLICE=1024 selects TAMD_SLICE_BYTES (tamd_exec16); fixed for the process.
extern const uint32_t g_slice_bytes;
inline uint32_t slice_bytes() { return g_slice_bytes; }
// Work items of an op spanning `span` bytes (at least one): constant divisors, no division.
inline uint32_t op_slices(uint32_t span) {
    const uint32_t n = g_slice_bytes == TAMD_SLICE_BYTES_X ? (span + TAMD_SLICE_BYTES_X - 1) / TAMD_SLICE_BYTES_X
                                                            : (span + TAMD_SLICE_BYTES - 1) / TAMD_SLICE_BYTES;
    return n ? n : 1u;
}

// ---------------------------------------------------------------------------------------------
// Arena bookkeeping: rows are contiguous ranges of 64-byte units in one device allocation.
// ---------------------------------------------------------------------------------------------
// Source of further arena segments for a RowTable that may grow (the siamese.h C ABI: one table
// per codec, segments handed out by a shared pool).  get() returns a free range of at least
// `min_units` 64-byte units (false when the arena cannot grow); put() takes a range back once no
// pending device work can touch it.
class SegmentSource {
public:
    virtual ~SegmentSource() {}
    virtual bool get(uint32_t min_units, uint64_t* base_units, uint32_t* units) = 0;
    virtual void put(uint64_t base_units, uint32_t units) = 0;
};

class RowTable {
public:
    ~RowTable();
    // Manage `bytes` of the device arena starting at 64-byte unit `base_units`.
    void init(uint64_t bytes, uint64_t base_units = 0);
    // Grow on demand: every range comes from `src` (none up front); returned to it on destruction.
    void init_segmented(SegmentSource* src);

    // Allocate a row with capacity >= bytes (rounded up to 64 B).  Returns kNoRow when full.
    RowId alloc(uint32_t bytes);
    // Release a row.  The memory is not reused until release_deferred() (called by the owner
    // once every program that may still read the row has completed on the device).
    void free_deferred(RowId r) {
        if (r != kNoRow) pending_.push_back(Pending{open_epoch_, r});
    }
    // Make rows freed since the previous call reusable.  `epoch` must be the flush epoch whose
    // device work has completed.
    void release_up_to(uint64_t completed_epoch);
    void seal_epoch(uint64_t epoch);  // rows freed so far belong to `epoch`

    uint32_t offset(RowId r) const { return off_[r]; }  // 64-B units from the arena base
    // Whether rows r0 .. r0 + k - 1 are live handles at offsets off(r0) + j * stride (a run of
    // rows laid out in order, as a session's inputs are): one contiguous scan of the offsets.
    bool affine(RowId r0, uint32_t k, uint32_t stride) const {
        if ((size_t)r0 + k > off_.size()) return false;
        const uint32_t* o = off_.data() + r0;
        const uint32_t o0 = o[0];
        uint32_t bad = 0;
        for (uint32_t j = 0; j < k; ++j) bad |= o[j] ^ (o0 + j * stride);
        return bad == 0;
    }
    uint32_t cap_bytes(RowId r) const { return units_[r] * TAMD_ROW_UNIT; }
    uint32_t units(RowId r) const { return units_[r]; }
    // Only rows written by the pending program have a level; a bitmap keeps the common case
    // (level 0) to one bit test instead of a lookup in the (large, cold) per-row tables.
    uint32_t level(RowId r) const { return ((hot_[r >> 6] >> (r & 63)) & 1u) ? level_[r] : 0u; }
    void set_level(RowId r, uint32_t l) {
        if (l) {
            hot_[r >> 6] |= 1ull << (r & 63);
            level_[r] = l;
        } else {
            hot_[r >> 6] &= ~(1ull << (r & 63));
        }
    }
    size_t live_rows() const { return live_; }
    uint64_t bytes_in_use() const { return (uint64_t)used_units_ * TAMD_ROW_UNIT; }
    // Keep the segments on destruction instead of returning them to the source: device work that
    // may still write them (a command that never completed) must not land in another codec's rows.
    void leak_segments() { src_ = nullptr; segments_.clear(); }

private:
    // per row handle (structure of arrays: offset lookups dominate)
    std::vector<uint32_t> off_, units_, level_;
    std::vector<uint64_t> hot_;  // bit per handle: level > 0
    std::vector<RowId> free_handles_;
    std::vector<std::vector<uint32_t>> free_offsets_;  // by size in units (small sizes)
    std::vector<std::pair<uint32_t, uint32_t>> free_big_; // (off, units) for large rows
    struct Pending { uint64_t epoch; RowId row; };
    std::vector<Pending> pending_;  // nondecreasing epochs; [pending_head_, end) not yet released
    size_t pending_head_ = 0;
    uint64_t open_epoch_ = 1;       // epoch rows freed now belong to
    uint32_t bump_ = 0, bump_end_ = 0;  // free tail of the current range (absolute units)
    SegmentSource* src_ = nullptr;
    std::vector<std::pair<uint64_t, uint32_t>> segments_;  // ranges taken from src_
    uint64_t used_units_ = 0;
    size_t live_ = 0;
    void release(RowId r);
};

// ---------------------------------------------------------------------------------------------
// Device program under construction.
// ---------------------------------------------------------------------------------------------
class ProgramBuilder {
public:
    explicit ProgramBuilder(RowTable* rows) : rows_(rows) {}

    // Emit `dst[0:len] = sum terms`, followed by `footer` (<= 8 bytes) and zero fill to the
    // row capacity.  Assigns and returns the op's level (also recorded on dst).
    uint32_t combine(RowId dst, const Term* terms, size_t n, uint32_t len,
                     const uint8_t* footer = nullptr, uint32_t footer_len = 0);

    // Raw op construction for scans: begin, add ACC/ACC3/STORE instructions, end.
    void begin_op();
    void op_acc(RowId src, uint8_t coef, uint32_t len, uint32_t acc = 0);
    void op_acc3_off(uint32_t off, uint8_t c1, uint8_t c2, uint32_t len);  // level-0 row at `off`
    // A strided run of level-0 rows (program.h ACCR); row0/stride in 64-B units.
    void op_accr(uint32_t mode, uint32_t param, uint32_t row0, uint32_t stride, uint32_t count, uint32_t len,
                 uint32_t col0, uint32_t cstep);
    // MULTI run: targets t[a] = kind | p << 8 | hi << 16 accumulate into acc_a (program.h).
    void op_accr_multi(uint32_t row0, uint32_t stride, uint32_t count, uint32_t len, uint32_t col0, uint32_t cstep,
                       const uint32_t t[3]);
    // DENSE run: a Siamese row's dense part over a run of level-0 packets (program.h); `ops` holds
    // the row's 8 lane opcodes, 6 bits each; adj[0..nadj) = (index in the run) << 16 | delta << 8
    // coefficient additions (ADJ words).
    void op_accr_dense(uint32_t row0, uint32_t stride, uint32_t count, uint32_t len, uint32_t col0, uint64_t ops,
                       uint8_t rx, const uint32_t* adj = nullptr, uint32_t nadj = 0, uint8_t scale = 1);
    // DENSE run for 2-3 rows at once (program.h): target t (COEFS word: lane opcodes `ops`, `rx`;
    // rows i < hi of the run; ADJ additions adj[0..nadj)) accumulates into acc_t.  The op stays a
    // shareable combine when it ends in op_store_shared stores only.
    struct DenseCoefs { uint64_t ops; uint8_t rx; uint32_t hi; const uint32_t* adj; uint32_t nadj; };
    void op_accr_dense_multi(uint32_t row0, uint32_t stride, uint32_t count, uint32_t len, uint32_t col0,
                             const DenseCoefs* t, uint32_t nt);
    // STORE (+FOOTER) of acc_a at the end of an op whose row batches waves may split: the executor
    // reduces each stored accumulator across the waves (at most three stores, the op's last words).
    void op_store_shared(RowId dst, uint32_t len, uint32_t acc, const uint8_t* footer, uint32_t footer_len);
    // Register a run of level-0 rows at offsets off0 + k * stride (k < count), columns col0 + k,
    // with per-row coefficients CauchyElement(p, column mod 64) (mode TAMD_R_CAUCHY) or 1
    // (TAMD_R_CONST), as one symbolic term (kRunFlag) of length len; combine() emits it as one
    // ACCR run scaled by the term's coefficient.  Valid until clear().
    Term run_term(uint32_t mode, uint32_t p, uint32_t off0, uint32_t stride, uint32_t count, uint32_t col0,
                  uint32_t len) {
        runs_.push_back(RunRef{mode, p, off0, stride, count, col0, 0, 0, 0});
        return Term{kRunFlag | (uint32_t)(runs_.size() - 1), len, 1};
    }
    // The same for a Siamese row's dense part over a run of level-0 packets (TAMD_R_DENSE: lane
    // opcodes `ops`, `rx`, coefficient additions adj[0..nadj) as op_accr_dense takes them): the
    // decoder's elimination of received originals straight from the packets.  combine() emits it
    // as one DENSE run scaled by the term's coefficient.
    Term dense_run_term(uint32_t off0, uint32_t stride, uint32_t count, uint32_t col0, uint64_t ops, uint8_t rx,
                        const uint32_t* adj, uint32_t nadj, uint32_t len) {
        const uint32_t at = (uint32_t)run_adj_.size();
        run_adj_.insert(run_adj_.end(), adj, adj + nadj);
        runs_.push_back(RunRef{TAMD_R_DENSE, rx, off0, stride, count, col0, ops, at, nadj});
        return Term{kRunFlag | (uint32_t)(runs_.size() - 1), len, 1};
    }
    // STORE (+FOOTER) of acc_0 into dst and close the op (the tail of combine()).
    uint32_t finish_combine(RowId dst, uint32_t len, const uint8_t* footer, uint32_t footer_len);
    void op_store(RowId dst, uint32_t len, uint32_t acc = 0, const uint8_t* footer = nullptr, uint32_t footer_len = 0);
    void op_storec(RowId dst, uint32_t len, const uint8_t* c);  // c0*acc_0 ^ c1*acc_1 ^ c2*acc_2
    // The same into a part of row `dst` (`units` 64-B units from its start, `cap` bytes); the
    // row is recorded as written once (`first`: the first part the op stores).
    void op_storec_part(RowId dst, uint32_t units, uint32_t len, uint32_t cap, const uint8_t* c, bool first);
    // ACC of a part of row `src` (its level is the row's).
    void op_acc_part(RowId src, uint32_t units, uint8_t coef, uint32_t len, uint32_t acc);
    uint32_t end_op(uint32_t min_level = 1);  // returns level; rows stored get that level

    bool empty() const { return ops_.empty(); }
    void clear();
    // Exchange the finished contents (no op may be under construction in either builder).
    void swap_contents(ProgramBuilder& o) {
        ops_.swap(o.ops_);
        instrs_.swap(o.instrs_);
        levels_.swap(o.levels_);
        pure_.swap(o.pure_);
        written_.swap(o.written_);
        level_ops_.swap(o.level_ops_);
        level_items_.swap(o.level_items_);
        std::swap(max_level_, o.max_level_);
        std::swap(acc_bytes_, o.acc_bytes_);
        std::swap(store_bytes_, o.store_bytes_);
    }
    uint32_t max_level() const { return max_level_; }

    const std::vector<tamd_op>& ops() const { return ops_; }
    const InstrVec& instrs() const { return instrs_; }
    // Per op: its bucket, TAMD_COST_CLASSES * level + cost class (0 = most expensive).
    const std::vector<uint32_t>& op_levels() const { return levels_; }
    // Per op: 1 when it is a pure combine (ACC into acc_0, CONST/CAUCHY/DENSE runs, one final
    // STORE + FOOTER) whose row batches several waves can split (partial sums reduced after);
    // 2 when it is such a combine into up to three accumulators (multi-target DENSE runs, one
    // STORE + FOOTER per accumulator).
    const std::vector<uint8_t>& op_pure() const { return pure_; }
    const std::vector<RowId>& written_rows() const { return written_; }
    // Per bucket (see op_levels): op count and work-item count (slice_bytes() chunks).
    const std::vector<uint32_t>& level_ops() const { return level_ops_; }
    const std::vector<uint32_t>& level_items() const { return level_items_; }

    uint64_t acc_bytes() const { return acc_bytes_; }       // sum of ACC lengths (op-trace)
    uint64_t store_bytes() const { return store_bytes_; }

private:
    RowTable* rows_;
    std::vector<tamd_op> ops_;
    InstrVec instrs_;
    std::vector<uint32_t> levels_;
    std::vector<uint8_t> pure_;
    std::vector<RowId> written_;
    std::vector<uint32_t> level_ops_, level_items_;
    uint32_t max_level_ = 0;
    // op under construction
    uint32_t cur_first_ = 0, cur_span_ = 0, cur_level_in_ = 0, cur_full_ = ~0u, cur_runs_ = 0;
    bool cur_pure_ = true;  // only acc_0 sums and CONST/CAUCHY runs so far (see TAMD_COST_CLASSES)
    bool cur_multi_ = false;  // (pure) multi-target DENSE runs: pure_ value 2
    struct RunRef { uint32_t mode, p, off0, stride, count, col0; uint64_t ops; uint32_t adj0, nadj; };
    std::vector<RunRef> runs_;  // run terms of the pending program
    std::vector<uint32_t> run_adj_;  // ADJ words of DENSE run terms
    size_t cur_written_begin_ = 0;
    uint64_t acc_bytes_ = 0, store_bytes_ = 0, cur_acc_begin_ = 0;
};

// ---------------------------------------------------------------------------------------------
// Term-list helpers (all lengths clip like the reference's byte counts).
// ---------------------------------------------------------------------------------------------
inline void sym_add(Sym& dst, const Term* src, size_t n, uint32_t limit, uint8_t coef = 1) {
    if (coef == 0) return;
    for (size_t i = 0; i < n; ++i) {
        Term t = src[i];
        if (t.len > limit) t.len = limit;
        if (t.len == 0) continue;
        t.coef = coef == 1 ? t.coef : gf_mul(t.coef, coef);
        if (t.coef) dst.push_back(t);
    }
}
inline void sym_add(Sym& dst, const Sym& src, uint32_t limit, uint8_t coef = 1) {
    sym_add(dst, src.data(), src.size(), limit, coef);
}
inline void sym_scale(Sym& s, uint8_t coef) {
    if (coef == 1) return;
    size_t k = 0;
    for (size_t i = 0; i < s.size(); ++i) {
        Term t = s[i];
        t.coef = gf_mul(t.coef, coef);
        if (t.coef) s[k++] = t;
    }
    s.resize(k);
}
inline void sym_clip(Sym& s, uint32_t limit) {
    size_t k = 0;
    for (size_t i = 0; i < s.size(); ++i) {
        Term t = s[i];
        if (t.len > limit) t.len = limit;
        if (t.len) s[k++] = t;
    }
    s.resize(k);
}
// Merge duplicate (row, len) terms, dropping cancelled ones.  Order is not significant.
void sym_merge(Sym& s);

// ---------------------------------------------------------------------------------------------
// The three running sums of one lane, as one scan.
//
// Sum s of a lane accumulates coef_s(cx) * row for every packet of the lane, where cx is the
// packet's column value and coef = (1, cx, cx^2) (SiameseEncoder.cpp:359-418,
// SiameseDecoder.cpp:1538-1739).  All three sums see the same packets in the same order, so
// the device walks them together: one ACC3 instruction per packet reads the row once and
// updates the three accumulators.  Recovery rows read the sums in fixed linear combinations
// (opcode bits select sums into the row and into the RX product), so a read is one snapshot
// row of c0*sum_0 + c1*sum_1 + c2*sum_2, written by a STOREC in the scan.
// ---------------------------------------------------------------------------------------------
class ExpansionTable;  // rows produced in the pending program -> their symbolic content

class LaneSums {
public:
    uint32_t bytes = 0;  // logical length, GrowingAlignedDataBuffer::Bytes semantics

    // Reference "Bytes = 0": the contents restart from zero.
    void reset(RowTable& rows);
    // GrowZeroPadded: only the logical length changes (data beyond is zero by construction).
    void grow(uint32_t b) { if (b > bytes) bytes = b; }
    // sum_s ^= cx^s * data for s = 0, 1, 2 (data = row, possibly produced in the pending program);
    // `column` is the packet number (cx = column_value(column)).  Consecutive lane packets whose
    // rows sit at a fixed stride are kept as one run (one ACCR on the device).
    void accumulate(RowTable& rows, RowId row, uint32_t len, uint32_t column) {
        if (!len) return;
        if (rows.level(row) != 0) {
            if (len > content_) content_ = len;
            dyn_.push_back(T{row, len, 0, 0, 1, column});
            return;
        }
        accumulate_level0(row, rows.offset(row), len, column);
    }
    // The same for a row known to be in memory already, at arena offset `off`.
    void accumulate_level0(RowId row, uint32_t off, uint32_t len, uint32_t column) {
        if (!len) return;
        if (len > content_) content_ = len;
        if (!terms_.empty()) {
            T& b = terms_.back();
            // (a run never wraps the 22-bit column period: the device steps cx by column)
            if (b.len == len && b.col + 8u * b.count == column) {
                if (b.count == 1 && off > b.off) {
                    b.stride = off - b.off;
                    b.count = 2;
                    ++n_;
                    return;
                }
                if (b.count > 1 && off == b.off + b.stride * b.count) {
                    ++b.count;
                    ++n_;
                    return;
                }
            }
        }
        terms_.push_back(T{row, len, off, 0, 1, column});
        ++n_;
    }
    // `count` level-0 lane packets at once: rows off + k * stride, columns column + 8k (the
    // same packets accumulate_level0 would take one by one; the run must not wrap the column
    // period).
    void accumulate_run_level0(RowId row, uint32_t off, uint32_t len, uint32_t column, uint32_t count,
                               uint32_t stride) {
        if (!len || !count) return;
        if (count == 1) {
            accumulate_level0(row, off, len, column);
            return;
        }
        if (len > content_) content_ = len;
        n_ += count;
        if (!terms_.empty()) {
            T& b = terms_.back();
            if (b.len == len && b.col + 8u * b.count == column) {
                if (b.count == 1 && off > b.off && off - b.off == stride) {
                    b.stride = stride;
                    b.count = 1 + count;
                    return;
                }
                if (b.count > 1 && b.stride == stride && off == b.off + b.stride * b.count) {
                    b.count += count;
                    return;
                }
            }
        }
        terms_.push_back(T{row, len, off, stride, count, column});
    }
    // Append c[0]*sum_0 + c[1]*sum_1 + c[2]*sum_2 (current values, clipped to `limit` bytes).
    // With `pb`, packets produced in this program that have piled up (dyn_, each read as its
    // expansion by every read) are first folded into three rows (dyn_fold_above()).
    // With `short_scan` (Context::short_scans), a snapshot taken while the scan is still one
    // op's length is promised the scan op's own level (1 over level-0 bases) instead of the chain
    // level, and the scan is then emitted as that one op.
    void read(RowTable& rows, const ExpansionTable& ex, Sym& out, const uint8_t* c, uint32_t limit,
              ProgramBuilder* pb = nullptr, bool short_scan = false);
    // Nothing accumulated since the last flush: a read only names the carried rows.
    bool idle() const { return terms_.empty() && dyn_.empty(); }
    // Emit the scan (and fix-up) ops for the pending program and rebase the sums.
    void flush(RowTable& rows, ProgramBuilder& pb, const ExpansionTable& ex);
    // Drop everything (codec destruction).
    void release(RowTable& rows);

private:
public:
    // a run of `count` lane packets: rows off + k*stride, columns col + 8k (count 1: a single row)
    struct T { RowId row; uint32_t len, off, stride, count, col; };
    static uint32_t chunk();  // longest packet walk of one scan op (see emit_scan)
    // read() folds dyn_ once it holds this many packets (TONK_AMD_DYN_FOLD; 0: never)
    static uint32_t dyn_fold_above();
    static uint32_t inline_max();  // segments this short are walked by the chain op (emit_scan)
    // Level of snapshot rows: chunk ops run at level 1, the chain op that stores the snapshots at
    // level 2 (a short scan is one op, also placed at level 2).  Readers are assigned levels when
    // they read, before the scan is emitted, so the level is fixed up front.
    static const uint32_t kSnapLevel = 2;
    // Level of a scan's snapshot rows over carried values `base` (kSnapLevel, or above the
    // bases when they are still being written: rows of this program or inherited ones).
    static uint32_t snap_level(const RowTable& rows, const RowId* base, uint32_t l = kSnapLevel) {
        for (unsigned s = 0; s < 3; ++s)
            if (base[s] != kNoRow && rows.level(base[s]) + 1 > l) l = rows.level(base[s]) + 1;
        return l;
    }

private:
    struct Snap { RowId row; uint32_t after; uint8_t c[3]; uint8_t level; };  // after = packets accumulated
    uint32_t n_ = 0;                            // packets in terms_
    RowId base_[3] = {kNoRow, kNoRow, kNoRow};  // carried values from a previous flush (level 0)
    uint32_t content_ = 0;                      // bytes the accumulated content may occupy
    std::vector<T> terms_;                      // level-0 packets accumulated since base_
    std::vector<Snap> snaps_;
    std::vector<T> dyn_;                        // packets produced in this program (level > 0)
    // dyn_ packets folded away: fold_[s] = sum over them of coef_s(cx) * packet (this program's
    // rows; read like base_, added into the carried values at flush)
    RowId fold_[3] = {kNoRow, kNoRow, kNoRow};
    uint32_t fold_len_ = 0;
    bool fold_dyn(RowTable& rows, ProgramBuilder& pb, const ExpansionTable& ex);
    void drop_fold(RowTable& rows);
    // closed epochs (reset while the program was pending) still owe their snapshots
    struct Closed { RowId base[3]; std::vector<T> terms; std::vector<Snap> snaps; };
    std::vector<Closed> closed_;  // [0, n_closed_) pending; the rest keep storage for reuse
    size_t n_closed_ = 0;
    static void emit_scan(RowTable& rows, ProgramBuilder& pb, const RowId* base, const std::vector<T>& terms,
                          const std::vector<Snap>& snaps, const RowId* final_rows);
};

inline uint8_t sum_coef(unsigned s, uint8_t cx) { return s == 0 ? 1 : (s == 1 ? cx : gf_sqr(cx)); }
// Coefficients of the lane sums a Siamese row reads (SiameseEncoder.cpp:1046-1098): opcode bit s
// adds sum s to the row, bit s + 3 adds it to the product that is multiplied by RX.
inline void opcode_coefs(unsigned op, uint8_t rx, uint8_t* c) {
    for (unsigned s = 0; s < 3; ++s)
        c[s] = (uint8_t)(((op >> s) & 1u) ^ (((op >> (s + 3)) & 1u) ? rx : 0u));
}

// Symbolic content of rows written by the pending program, so readers in the same flush can
// use the content's terms instead of the row itself (which would add a level).
class ExpansionTable {
public:
    // Expansions longer than this many terms are not inlined: the reader takes the row itself and
    // lands one level above its writer.  Unlimited by default (flat programs: one launch per
    // level); a pipelined session, whose levels overlap across programs, bounds it (the cost of
    // inlining grows with the solves per program).
    uint32_t expand_limit = ~0u;
    void set(RowId r, const Sym& s);
    // set() by exchanging storage: `s` is left with unspecified contents
    void take(RowId r, Sym& s);
    bool has(RowId r) const { return r < index_.size() && index_[r] >= 0; }
    const Sym& get(RowId r) const { return pool_[index_[r]]; }
    void clear();
    // Append `coef * content(r)[0:len]` to out: the row itself when it is already in memory
    // (level 0), otherwise its expansion.
    void append(const RowTable& rows, RowId r, uint32_t len, uint8_t coef, Sym& out) const;

private:
    std::vector<int32_t> index_;
    std::vector<Sym> pool_;  // [0, n_pool_) in use
    size_t n_pool_ = 0;
    std::vector<RowId> used_;
};

// Split a symbolic value: fold every term whose row level is below `keep_level` into a new
// row (a "partial", materialized by one combine op) and keep the rest symbolic.  Returns the
// new row or kNoRow when nothing was folded.
RowId fold_low_levels(RowTable& rows, ProgramBuilder& pb, Sym& s, uint32_t keep_level,
                      uint32_t len, uint32_t row_bytes);

// ---------------------------------------------------------------------------------------------
// Context: one arena range + one pending program.  Codecs attached to a context contribute to
// the same program; a flush hands the program to the executor and rebases every codec.
// ---------------------------------------------------------------------------------------------
class FlushClient {
public:
    virtual ~FlushClient() {}
    virtual void pre_flush() = 0;   // emit pending scans (running sums) into the program
    virtual void post_flush() = 0;  // drop per-program symbolic state
    bool dirty = false;              // on Context::dirty (touched since the last flush)
};

struct Context {
    RowTable rows;
    ProgramBuilder pb{&rows};
    // The last program closed by finish_flush(true): kept for the executor while the next one
    // is built (the session fills a program during the next step's control plane).
    ProgramBuilder closed{&rows};
    ExpansionTable ex;
    std::vector<RowId> temps;          // rows only read inside the pending program
    std::vector<FlushClient*> clients;
    uint64_t epoch = 1;                // id of the pending program
    uint64_t arena_base_units = 0;     // offset of this context's range in the device arena
    bool oom = false;                  // arena exhausted (codecs go to Disabled)
    // Decoder back substitution over materialized eliminated rows from this many unknowns on
    // (Decoder::back_substitution; ~0u: never).  Few-stream sessions use it; in batched ones the
    // extra level costs launches and saves no device bytes.
    uint32_t backsub_rows = ~0u;
    // Direct dense ranges longer than this are split into partial sums over two levels
    // (Encoder::defer_dense; 0: never).  Only batched sessions split: there a long op is a
    // launch's tail, while per-call programs (the C ABI) and single streams pay an extra level
    // launch in latency and already share a long op across a workgroup.
    uint32_t dense_split = 0;
    // Decoder eliminations of received originals from Siamese rows straight from the packets
    // (Decoder::eliminate_direct) where the row's sum range is short and made of long runs, as the
    // encoder's direct dense ranges; false: always through the decoder's lane sums.
    bool direct_elim = default_direct_elim();
    static bool default_direct_elim() {  // (TONK_AMD_DEC_DIRECT=0: A/B against the lanes)
        static const bool on = !(getenv("TONK_AMD_DEC_DIRECT") && atoi(getenv("TONK_AMD_DEC_DIRECT")) == 0);
        return on;
    }
    // Lane-sum snapshots read while a scan is one op long take that op's level (LaneSums::read):
    // per-call programs (the C ABI) flush right after their reads, so their scans stay short and
    // a Siamese recovery row lands one level earlier.
    bool short_scans = false;
    // Level pipelining (the session, Device::set_pipelined): every launch runs level 1 of the
    // newest program beside the next level of each older program still in flight, so level d
    // of a program runs with level 1 of the program d - 1 later.  A row written at level d is
    // therefore still being written while the next program's levels 1 .. d - 1 run: there it
    // keeps level d - 1 ("inherited", one less per program), and its readers land above it.
    static const uint32_t kPipeDepth = 1;
    bool pipeline = false;
    std::vector<RowId> inherited;      // rows with an inherited level in the pending program
    std::vector<uint64_t> written_mark;  // bitmap over handles, all zero between flushes

    RowId alloc(uint32_t bytes) {
        const RowId r = rows.alloc(bytes);
        if (r == kNoRow) oom = true;
        return r;
    }
    RowId alloc_temp(uint32_t bytes) {
        const RowId r = alloc(bytes);
        if (r != kNoRow) temps.push_back(r);
        return r;
    }
    void attach(FlushClient* c) { clients.push_back(c); }
    void detach(FlushClient* c) {
        clients.erase(std::remove(clients.begin(), clients.end(), c), clients.end());
        dirty.erase(std::remove(dirty.begin(), dirty.end(), c), dirty.end());
    }
    // Dirty tracking for contexts shared by many codecs (the siamese.h C ABI): a codec only has
    // pending scans after a call on it, so a flush visits the codecs touched since the last one
    // instead of every attached codec.  Off (every client visited) unless enabled.
    bool track_dirty = false;
    std::vector<FlushClient*> dirty;
    void touch(FlushClient* c) {
        if (!c->dirty) {
            c->dirty = true;
            dirty.push_back(c);
        }
    }
    // Close the pending program: scans emitted, temps released after `epoch` completes.  The
    // caller then executes pb's ops and calls finish_flush().
    void prepare_flush() {
        for (FlushClient* c : track_dirty ? dirty : clients) c->pre_flush();
    }
    void finish_flush(bool keep_closed = false) {
        const std::vector<RowId>& w = pb.written_rows();
        if (pipeline) {
            // Inherited entries of earlier programs count down one level (a row written at level
            // d stays pending d - 1 programs); a row written again now is superseded by its new
            // entry (a handle rewritten, or freed and reused while it was counting down).  The
            // rows written now are marked in a bitmap for that test: a per-handle epoch array
            // costs a cache miss per written row.
            if (!inherited.empty()) {
                for (RowId r : w) {
                    if ((r >> 6) >= written_mark.size()) written_mark.resize((r >> 6) + 1024, 0);
                    written_mark[r >> 6] |= 1ull << (r & 63);
                }
                size_t keep = 0;
                for (RowId r : inherited) {
                    if ((r >> 6) < written_mark.size() && ((written_mark[r >> 6] >> (r & 63)) & 1u)) continue;
                    const uint32_t l = rows.level(r);
                    if (l > kPipeDepth) {
                        rows.set_level(r, l - kPipeDepth);
                        inherited[keep++] = r;
                    } else {
                        rows.set_level(r, 0);
                    }
                }
                inherited.resize(keep);
                for (RowId r : w) written_mark[r >> 6] = 0;
            }
            for (RowId r : w) {
                const uint32_t l = rows.level(r);
                if (l > kPipeDepth) {
                    rows.set_level(r, l - kPipeDepth);
                    inherited.push_back(r);
                } else {
                    rows.set_level(r, 0);
                }
            }
        } else {
            for (RowId r : w) rows.set_level(r, 0);
        }
        for (RowId r : temps) rows.free_deferred(r);
        temps.clear();
        ex.clear();
        for (FlushClient* c : track_dirty ? dirty : clients) c->post_flush();
        for (FlushClient* c : dirty) c->dirty = false;
        dirty.clear();
        rows.seal_epoch(epoch);
        ++epoch;
        if (keep_closed) closed.swap_contents(pb);
        pb.clear();
    }
};

} // namespace tamd
