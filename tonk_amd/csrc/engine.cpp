// engine.cpp -- see engine.h.
#include "engine.h"

#include <stdio.h>
#include "prof.h"

#include <stdlib.h>
#include <string.h>

namespace tamd {

static uint32_t slice_from_env() {
    const char* e = getenv("TONK_AMD_SLICE");
    return e && atoi(e) == (int)TAMD_SLICE_BYTES ? TAMD_SLICE_BYTES : TAMD_SLICE_BYTES_X;
}
const uint32_t g_slice_bytes = slice_from_env();

// ---------------------------------------------------------------------------------------------
// RowTable
// ---------------------------------------------------------------------------------------------
static const uint32_t kSmallClasses = 256;  // rows up to 16 KB use exact-size free lists

RowTable::~RowTable() {
    if (src_)
        for (const auto& s : segments_) src_->put(s.first, s.second);
}

void RowTable::init(uint64_t arena_bytes, uint64_t base_units) {
    const uint64_t units = arena_bytes / TAMD_ROW_UNIT;
    uint64_t end = base_units + units;
    if (end > 0xfffffff0ull) end = 0xfffffff0ull;  // 32-bit unit offsets: 256 GiB of arena
    bump_ = (uint32_t)base_units;
    bump_end_ = (uint32_t)end;
    src_ = nullptr;
    segments_.clear();
    used_units_ = 0;
    live_ = 0;
    off_.clear();
    units_.clear();
    level_.clear();
    hot_.clear();
    free_handles_.clear();
    free_offsets_.assign(kSmallClasses + 1, std::vector<uint32_t>());
    free_big_.clear();
    pending_.clear();
    pending_head_ = 0;
    open_epoch_ = 1;
}

RowId RowTable::alloc(uint32_t bytes) {
    TAMD_PROF_SCOPE(kAlloc);
    uint32_t units = (bytes + TAMD_ROW_UNIT - 1) / TAMD_ROW_UNIT;
    if (units == 0) units = 1;
    uint32_t off = 0xffffffffu;
    if (units <= kSmallClasses && !free_offsets_[units].empty()) {
        off = free_offsets_[units].back();
        free_offsets_[units].pop_back();
    } else if (units > kSmallClasses) {
        for (size_t i = 0; i < free_big_.size(); ++i) {
            if (free_big_[i].second == units) {
                off = free_big_[i].first;
                free_big_[i] = free_big_.back();
                free_big_.pop_back();
                break;
            }
        }
    }
    if (off == 0xffffffffu) {
        if ((uint64_t)bump_ + units > bump_end_) {
            uint64_t base = 0;
            uint32_t got = 0;
            if (!src_ || !src_->get(units, &base, &got) || got < units || base + got > 0xfffffff0ull) return kNoRow;
            segments_.push_back(std::make_pair(base, got));
            // the old range's tail stays unused (rows are exact-size; tails are small)
            bump_ = (uint32_t)base;
            bump_end_ = (uint32_t)(base + got);
        }
        off = bump_;
        bump_ += units;
    }
    RowId h;
    if (!free_handles_.empty()) {
        h = free_handles_.back();
        free_handles_.pop_back();
    } else {
        h = (RowId)off_.size();
        off_.push_back(0);
        units_.push_back(0);
        level_.push_back(0);
        if ((h & 63) == 0) hot_.push_back(0);
    }
    off_[h] = off;
    units_[h] = units;
    hot_[h >> 6] &= ~(1ull << (h & 63));
    used_units_ += units;
    ++live_;
    return h;
}

void RowTable::init_segmented(SegmentSource* src) {
    init(0, 0);
    src_ = src;
}

void RowTable::release(RowId r) {
    const uint32_t units = units_[r], off = off_[r];
    if (units <= kSmallClasses) free_offsets_[units].push_back(off);
    else free_big_.push_back(std::make_pair(off, units));
    used_units_ -= units;
    --live_;
    free_handles_.push_back(r);
}

void RowTable::seal_epoch(uint64_t epoch) { open_epoch_ = epoch + 1; }

void RowTable::release_up_to(uint64_t completed) {
    size_t i = pending_head_;
    const size_t n = pending_.size();
    while (i < n && pending_[i].epoch <= completed) release(pending_[i++].row);
    if (i == n) {
        pending_.clear();
        pending_head_ = 0;
    } else if (i > 4096 && i * 2 > n) {
        pending_.erase(pending_.begin(), pending_.begin() + (std::ptrdiff_t)i);
        pending_head_ = 0;
    } else {
        pending_head_ = i;
    }
}

// ---------------------------------------------------------------------------------------------
// ProgramBuilder
// ---------------------------------------------------------------------------------------------
static void push_store(InstrVec& v, uint32_t off, uint32_t len, uint32_t cap,
                       const uint8_t* footer, uint32_t flen, uint32_t acc = 0);
void ProgramBuilder::clear() {
    ops_.clear();
    instrs_.clear();
    levels_.clear();
    pure_.clear();
    written_.clear();
    level_ops_.clear();
    level_items_.clear();
    runs_.clear();
    run_adj_.clear();
    max_level_ = 0;
    acc_bytes_ = store_bytes_ = 0;
}

void ProgramBuilder::begin_op() {
    cur_acc_begin_ = acc_bytes_;
    cur_first_ = (uint32_t)instrs_.size();
    cur_span_ = 0;
    cur_full_ = ~0u;
    cur_runs_ = 0;
    cur_pure_ = true;
    cur_multi_ = false;
    cur_level_in_ = 0;
    cur_written_begin_ = written_.size();
}

void ProgramBuilder::op_acc3_off(uint32_t off, uint8_t c1, uint8_t c2, uint32_t len) {
    if (!len) return;
    tamd_instr in;
    cur_pure_ = false;
    in.w0 = tamd_w0(TAMD_I_ACC3, c1, c2);
    in.row = off;
    in.len = len;
    in.cap = 0;
    instrs_.push_back(in);
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    acc_bytes_ += len;
}

void ProgramBuilder::op_accr(uint32_t mode, uint32_t param, uint32_t row0, uint32_t stride, uint32_t count,
                             uint32_t len, uint32_t col0, uint32_t cstep) {
    if (!len || !count) return;
    tamd_instr a, r;
    a.w0 = tamd_w0(TAMD_I_ACCR, mode, param);
    a.row = row0;
    a.len = len;
    a.cap = count;
    r.w0 = TAMD_I_RANGE;
    r.row = stride;
    r.len = col0;
    r.cap = cstep;
    instrs_.push_back(a);
    instrs_.push_back(r);
    ++cur_runs_;
    if (mode == TAMD_R_LANE3) cur_pure_ = false;
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    acc_bytes_ += (uint64_t)len * count;
}

void ProgramBuilder::op_accr_multi(uint32_t row0, uint32_t stride, uint32_t count, uint32_t len, uint32_t col0,
                                   uint32_t cstep, const uint32_t t[3]) {
    if (!len || !count) return;
    tamd_instr a, r, g;
    a.w0 = tamd_w0(TAMD_I_ACCR, TAMD_R_MULTI, 0);
    a.row = row0;
    a.len = len;
    a.cap = count;
    r.w0 = TAMD_I_RANGE;
    r.row = stride;
    r.len = col0;
    r.cap = cstep;
    g.w0 = TAMD_I_TARGETS;
    g.row = t[0];
    g.len = t[1];
    g.cap = t[2];
    instrs_.push_back(a);
    instrs_.push_back(r);
    instrs_.push_back(g);
    ++cur_runs_;
    cur_pure_ = false;
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    acc_bytes_ += (uint64_t)len * count;
}

void ProgramBuilder::op_accr_dense(uint32_t row0, uint32_t stride, uint32_t count, uint32_t len, uint32_t col0,
                                   uint64_t ops, uint8_t rx, const uint32_t* adj, uint32_t nadj, uint8_t scale) {
    if (!len || !count || !scale) return;
    const uint32_t nwords = (nadj + 3) / 4;
    tamd_instr a, r, g;
    a.w0 = tamd_w0(TAMD_I_ACCR, TAMD_R_DENSE, 0) | (scale > 1 ? (uint32_t)scale << 24 : 0u);
    a.row = row0;
    a.len = len;
    a.cap = count;
    r.w0 = TAMD_I_RANGE;
    r.row = stride;
    r.len = col0;
    r.cap = 1;
    g.w0 = TAMD_I_COEFS;
    g.row = (uint32_t)ops;
    g.len = (uint32_t)(ops >> 32) & 0xffffu;
    g.len |= (uint32_t)rx << 16;
    g.cap = nwords;
    instrs_.push_back(a);
    instrs_.push_back(r);
    instrs_.push_back(g);
    for (uint32_t w = 0; w < nwords; ++w) {
        uint32_t d[4] = {0, 0, 0, 0};
        for (uint32_t q = 0; q < 4 && 4 * w + q < nadj; ++q) d[q] = adj[4 * w + q];
        tamd_instr x;
        x.w0 = (d[0] & ~0xffu) | TAMD_I_ADJ;
        x.row = d[1];
        x.len = d[2];
        x.cap = d[3];
        instrs_.push_back(x);
    }
    ++cur_runs_;  // (acc_0 only: the op stays a pure combine)
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    acc_bytes_ += (uint64_t)len * count;
}

void ProgramBuilder::op_accr_dense_multi(uint32_t row0, uint32_t stride, uint32_t count, uint32_t len,
                                         uint32_t col0, const DenseCoefs* t, uint32_t nt) {
    if (!len || !count || nt < 2 || nt > 3) return;
    tamd_instr a, r;
    a.w0 = tamd_w0(TAMD_I_ACCR, TAMD_R_DENSE, nt);
    a.row = row0;
    a.len = len;
    a.cap = count;
    r.w0 = TAMD_I_RANGE;
    r.row = stride;
    r.len = col0;
    r.cap = 1;
    instrs_.push_back(a);
    instrs_.push_back(r);
    for (uint32_t k = 0; k < nt; ++k) {
        const uint32_t nwords = (t[k].nadj + 3) / 4;
        tamd_instr g;
        g.w0 = TAMD_I_COEFS;
        g.row = (uint32_t)t[k].ops;
        g.len = ((uint32_t)(t[k].ops >> 32) & 0xffffu) | (uint32_t)t[k].rx << 16;
        g.cap = nwords | (t[k].hi < count ? t[k].hi : count) << 16;
        instrs_.push_back(g);
        for (uint32_t w = 0; w < nwords; ++w) {
            uint32_t d[4] = {0, 0, 0, 0};
            for (uint32_t q = 0; q < 4 && 4 * w + q < t[k].nadj; ++q) d[q] = t[k].adj[4 * w + q];
            tamd_instr x;
            x.w0 = (d[0] & ~0xffu) | TAMD_I_ADJ;
            x.row = d[1];
            x.len = d[2];
            x.cap = d[3];
            instrs_.push_back(x);
        }
    }
    ++cur_runs_;
    cur_multi_ = true;
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    acc_bytes_ += (uint64_t)len * count;
}

void ProgramBuilder::op_store_shared(RowId dst, uint32_t len, uint32_t acc, const uint8_t* footer,
                                     uint32_t footer_len) {
    const uint32_t cap = rows_->cap_bytes(dst);
    push_store(instrs_, rows_->offset(dst), len, cap, footer, footer_len, acc);
    if (acc) cur_multi_ = true;
    if (cap > cur_span_) cur_span_ = cap;
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    written_.push_back(dst);
    store_bytes_ += len + footer_len;
}

uint32_t ProgramBuilder::finish_combine(RowId dst, uint32_t len, const uint8_t* footer, uint32_t footer_len) {
    const uint32_t cap = rows_->cap_bytes(dst);
    push_store(instrs_, rows_->offset(dst), len, cap, footer, footer_len);
    if (cap > cur_span_) cur_span_ = cap;
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    written_.push_back(dst);
    store_bytes_ += len + footer_len;
    return end_op(1);
}

void ProgramBuilder::op_acc(RowId src, uint8_t coef, uint32_t len, uint32_t acc) {
    if (!coef || !len) return;
    tamd_instr in;
    if (acc != 0) cur_pure_ = false;
    in.w0 = tamd_w0(TAMD_I_ACC, coef, acc);
    in.row = rows_->offset(src);
    in.len = len;
    in.cap = 0;
    instrs_.push_back(in);
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    const uint32_t l = rows_->level(src);
    if (l > cur_level_in_) cur_level_in_ = l;
    acc_bytes_ += len;
}

static void push_store(InstrVec& v, uint32_t off, uint32_t len, uint32_t cap,
                       const uint8_t* footer, uint32_t flen, uint32_t acc) {
    tamd_instr s;
    s.w0 = tamd_w0(TAMD_I_STORE, flen, acc);
    s.row = off;
    s.len = len;
    s.cap = cap;
    v.push_back(s);
    tamd_instr f;
    uint8_t fb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (flen) memcpy(fb, footer, flen);
    f.w0 = tamd_w0(TAMD_I_FOOTER, 0);
    memcpy(&f.row, fb, 4);
    memcpy(&f.len, fb + 4, 4);
    f.cap = 0;
    v.push_back(f);
}

void ProgramBuilder::op_storec(RowId dst, uint32_t len, const uint8_t* c) {
    const uint32_t cap = rows_->cap_bytes(dst);
    tamd_instr s;
    cur_pure_ = false;
    s.w0 = TAMD_I_STOREC | ((uint32_t)c[0] << 8) | ((uint32_t)c[1] << 16) | ((uint32_t)c[2] << 24);
    s.row = rows_->offset(dst);
    s.len = len;
    s.cap = cap;
    instrs_.push_back(s);
    if (cap > cur_span_) cur_span_ = cap;
    if (len < cur_full_) cur_full_ = len;
    written_.push_back(dst);
    store_bytes_ += len;
}

void ProgramBuilder::op_storec_part(RowId dst, uint32_t units, uint32_t len, uint32_t cap, const uint8_t* c,
                                    bool first) {
    tamd_instr s;
    cur_pure_ = false;
    s.w0 = TAMD_I_STOREC | ((uint32_t)c[0] << 8) | ((uint32_t)c[1] << 16) | ((uint32_t)c[2] << 24);
    s.row = rows_->offset(dst) + units;
    s.len = len;
    s.cap = cap;
    instrs_.push_back(s);
    if (cap > cur_span_) cur_span_ = cap;
    if (len < cur_full_) cur_full_ = len;
    if (first) written_.push_back(dst);
    store_bytes_ += len;
}

void ProgramBuilder::op_acc_part(RowId src, uint32_t units, uint8_t coef, uint32_t len, uint32_t acc) {
    if (!coef || !len) return;
    tamd_instr in;
    if (acc != 0) cur_pure_ = false;
    in.w0 = tamd_w0(TAMD_I_ACC, coef, acc);
    in.row = rows_->offset(src) + units;
    in.len = len;
    in.cap = 0;
    instrs_.push_back(in);
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    const uint32_t l = rows_->level(src);
    if (l > cur_level_in_) cur_level_in_ = l;
    acc_bytes_ += len;
}

void ProgramBuilder::op_store(RowId dst, uint32_t len, uint32_t acc, const uint8_t* footer, uint32_t footer_len) {
    cur_pure_ = false;  // (pure combines end with finish_combine / combine only)
    const uint32_t cap = rows_->cap_bytes(dst);
    push_store(instrs_, rows_->offset(dst), len, cap, footer, footer_len, acc);
    if (cap > cur_span_) cur_span_ = cap;
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    written_.push_back(dst);
    store_bytes_ += len + footer_len;
}

uint32_t ProgramBuilder::end_op(uint32_t min_level) {
    uint32_t level = cur_level_in_ + 1;
    if (level < min_level) level = min_level;
    tamd_op op;
    op.first = cur_first_;
    op.count = (uint32_t)instrs_.size() - cur_first_;
    op.span = (cur_span_ + 7u) & ~7u;
    op.full = cur_full_ < op.span ? cur_full_ : op.span;
    ops_.push_back(op);
    // Cost class from the op's length in the executor's terms: instructions, and row loads
    // (an ACCR run is `count` rows); class 0 is the most expensive and starts first.
    // (TONK_AMD_CLASS="rows_div,t1,t2,t3,rows0": A/B knob for the thresholds, default 2,64,32,12,48)
    struct ClassCfg {
        uint64_t div = 2, t1 = 64, t2 = 32, t3 = 12, r0 = 48;
        ClassCfg() {
            if (const char* e = getenv("TONK_AMD_CLASS")) {
                unsigned long long v[5] = {div, t1, t2, t3, r0};
                sscanf(e, "%llu,%llu,%llu,%llu,%llu", &v[0], &v[1], &v[2], &v[3], &v[4]);
                div = v[0] ? v[0] : 2;
                t1 = v[1];
                t2 = v[2];
                t3 = v[3];
                r0 = v[4];
            }
        }
    };
    static const ClassCfg cc;
    const uint64_t rows = (acc_bytes_ - cur_acc_begin_) / 1024u;
    const uint64_t cost = op.count + 4u * cur_runs_ + rows / cc.div;
    const uint32_t cls = (cur_pure_ && rows >= cc.r0) ? 0u : cost >= cc.t1 ? 1u : cost >= cc.t2 ? 2u : cost >= cc.t3 ? 3u : 4u;
    const uint32_t bucket = TAMD_COST_CLASSES * level + cls;
    levels_.push_back(bucket);
    pure_.push_back(cur_pure_ ? (cur_multi_ ? 2 : 1) : 0);
    if (level_ops_.size() < TAMD_COST_CLASSES * (level + 1)) {
        level_ops_.resize(TAMD_COST_CLASSES * (level + 1), 0);
        level_items_.resize(TAMD_COST_CLASSES * (level + 1), 0);
    }
    level_ops_[bucket]++;
    level_items_[bucket] += op_slices(op.span);
    for (size_t i = cur_written_begin_; i < written_.size(); ++i) rows_->set_level(written_[i], level);
    if (level > max_level_) max_level_ = level;
    return level;
}

uint32_t ProgramBuilder::combine(RowId dst, const Term* terms, size_t n, uint32_t len,
                                 const uint8_t* footer, uint32_t footer_len) {
    TAMD_PROF_SCOPE(kCombine);
    begin_op();
    // inline op_acc over the term list: one resize, then straight stores
    const size_t at = instrs_.size();
    instrs_.resize(at + n);
    tamd_instr* w = instrs_.data() + at;
    uint32_t span = cur_span_, lvl = cur_level_in_, full = cur_full_;
    uint64_t acc = 0;
    size_t k = 0, nrun = 0;
    for (size_t i = 0; i < n; ++i) {
        const Term& t = terms[i];
        if (!t.coef || !t.len) continue;
        if (is_run(t.row)) {
            ++nrun;
            continue;
        }
        w[k].w0 = tamd_w0(TAMD_I_ACC, t.coef);
        w[k].row = rows_->offset(t.row);
        w[k].len = t.len;
        w[k].cap = 0;
        ++k;
        if (t.len > span) span = t.len;
        if (t.len < full) full = t.len;
        const uint32_t l = rows_->level(t.row);
        if (l > lvl) lvl = l;
        acc += t.len;
    }
    instrs_.resize(at + k);
    cur_span_ = span;
    cur_full_ = full;
    cur_level_in_ = lvl;
    acc_bytes_ += acc;
    for (size_t i = 0; nrun && i < n; ++i) {
        const Term& t = terms[i];
        if (!t.coef || !t.len || !is_run(t.row)) continue;
        const RunRef& r = runs_[t.row & ~kRunFlag];
        --nrun;
        if (r.mode == TAMD_R_DENSE) {  // (its scale rides in the ACCR word)
            op_accr_dense(r.off0, r.stride, r.count, t.len, r.col0, r.ops, (uint8_t)r.p, run_adj_.data() + r.adj0,
                          r.nadj, t.coef);
            continue;
        }
        // a CONST run's constant is the coefficient itself; a CAUCHY run carries it as its scale
        const uint32_t param = r.mode == TAMD_R_CONST ? gf_mul((uint8_t)r.p, t.coef) : r.p | (uint32_t)t.coef << 8;
        op_accr(r.mode, param, r.off0, r.stride, r.count, t.len, r.col0, 1);
    }
    const uint32_t cap = rows_->cap_bytes(dst);
    push_store(instrs_, rows_->offset(dst), len, cap, footer, footer_len);
    if (cap > cur_span_) cur_span_ = cap;
    if (len > cur_span_) cur_span_ = len;
    if (len < cur_full_) cur_full_ = len;
    written_.push_back(dst);
    store_bytes_ += len + footer_len;
    return end_op(1);
}

// ---------------------------------------------------------------------------------------------
// Term lists
// ---------------------------------------------------------------------------------------------
void sym_merge(Sym& s) {
    const size_t n = s.size();
    if (n < 2) return;
    TAMD_PROF_SCOPE(kSymMerge);
    size_t k = 0;
    if (n <= 16) {
        for (size_t i = 0; i < n; ++i) {
            const Term t = s[i];
            size_t j = 0;
            while (j < k && (s[j].row != t.row || s[j].len != t.len)) ++j;
            if (j < k) s[j].coef ^= t.coef;
            else s[k++] = t;
        }
    } else {
        // open addressing on the row id; slots hold output positions (< the input position) and
        // are valid only when stamped with this call's generation (no clearing between calls)
        struct Slot { uint32_t gen; int32_t at; };
        thread_local std::vector<Slot> tab;
        thread_local uint32_t gen = 0;
        size_t cap = 32;
        while (cap < 2 * n) cap *= 2;
        if (tab.size() < cap) {
            tab.assign(cap, Slot{0, -1});
            gen = 0;
        }
        if (++gen == 0) {
            for (Slot& sl : tab) sl.gen = 0;
            gen = 1;
        }
        const size_t mask = cap - 1;
        for (size_t i = 0; i < n; ++i) {
            const Term t = s[i];
            size_t h = ((size_t)t.row * 0x9E3779B1u) >> 7 & mask;
            for (;;) {
                Slot& sl = tab[h];
                if (sl.gen != gen) {
                    sl.gen = gen;
                    sl.at = (int32_t)k;
                    s[k++] = t;
                    break;
                }
                const int32_t at = sl.at;
                if (s[at].row == t.row && s[at].len == t.len) {
                    s[at].coef ^= t.coef;
                    break;
                }
                h = (h + 1) & mask;
            }
        }
    }
    size_t m = 0;
    for (size_t i = 0; i < k; ++i)
        if (s[i].coef) s[m++] = s[i];
    s.resize(m);
}

// ---------------------------------------------------------------------------------------------
// ExpansionTable
// ---------------------------------------------------------------------------------------------
void ExpansionTable::set(RowId r, const Sym& s) {
    if (r >= index_.size()) index_.resize((size_t)r + 1, -1);
    if (index_[r] >= 0) { pool_[index_[r]] = s; return; }
    index_[r] = (int32_t)n_pool_;
    // pool entries keep their storage across programs (no allocation per expansion)
    if (n_pool_ < pool_.size()) pool_[n_pool_].assign(s.begin(), s.end());
    else pool_.push_back(s);
    ++n_pool_;
    used_.push_back(r);
}

void ExpansionTable::take(RowId r, Sym& s) {
    if (r >= index_.size()) index_.resize((size_t)r + 1, -1);
    if (index_[r] >= 0) { pool_[index_[r]].swap(s); return; }
    index_[r] = (int32_t)n_pool_;
    if (n_pool_ == pool_.size()) pool_.emplace_back();
    pool_[n_pool_].swap(s);
    ++n_pool_;
    used_.push_back(r);
}

void ExpansionTable::clear() {
    for (RowId r : used_) index_[r] = -1;
    used_.clear();
    n_pool_ = 0;
}

void ExpansionTable::append(const RowTable& rows, RowId r, uint32_t len, uint8_t coef, Sym& out) const {
    if (!coef || !len) return;
    if (rows.level(r) == 0 || !has(r) || get(r).size() > expand_limit) {
        out.push_back(Term{r, len, coef});
        return;
    }
    sym_add(out, get(r), len, coef);
}

// ---------------------------------------------------------------------------------------------
// LaneSums
// ---------------------------------------------------------------------------------------------
uint32_t LaneSums::chunk() {
    static const uint32_t c = getenv("TONK_AMD_CHUNK") ? (uint32_t)atoi(getenv("TONK_AMD_CHUNK")) : 64u;  // A/B
    return c ? c : 64u;
}

void LaneSums::reset(RowTable& rows) {
    if (!snaps_.empty()) {
        // Closed entries are reused across flushes: the swap hands this scan's lists to the entry
        // and takes back the storage of an earlier one, so neither side reallocates as it grows.
        if (n_closed_ == closed_.size()) closed_.emplace_back();
        Closed& c = closed_[n_closed_++];
        for (unsigned s = 0; s < 3; ++s) c.base[s] = base_[s];
        c.terms.swap(terms_);
        c.snaps.swap(snaps_);
    } else {
        for (unsigned s = 0; s < 3; ++s) rows.free_deferred(base_[s]);
    }
    for (unsigned s = 0; s < 3; ++s) base_[s] = kNoRow;
    terms_.clear();
    n_ = 0;
    snaps_.clear();
    dyn_.clear();
    drop_fold(rows);
    content_ = 0;
    bytes = 0;
}

static inline bool same_coefs(const uint8_t* a, const uint8_t* b) {
    return a[0] == b[0] && a[1] == b[1] && a[2] == b[2];
}

uint32_t LaneSums::dyn_fold_above() {
    static const uint32_t v = getenv("TONK_AMD_DYN_FOLD") ? (uint32_t)atoi(getenv("TONK_AMD_DYN_FOLD")) : 2u;
    return v;
}

// The dyn_ packets (and an earlier fold) into three rows, one combine each: every later read
// names those three rows instead of every packet's expansion again.
bool LaneSums::fold_dyn(RowTable& rows, ProgramBuilder& pb, const ExpansionTable& ex) {
    uint32_t len = fold_len_;
    for (const T& d : dyn_)
        if (d.len > len) len = d.len;
    RowId nf[3];
    for (unsigned s = 0; s < 3; ++s) {
        nf[s] = rows.alloc(len);
        if (nf[s] == kNoRow) {
            for (unsigned q = 0; q < s; ++q) rows.free_deferred(nf[q]);
            return false;
        }
    }
    thread_local Sym t;
    for (unsigned s = 0; s < 3; ++s) {
        t.clear();
        if (fold_[s] != kNoRow) t.push_back(Term{fold_[s], fold_len_, 1});
        for (const T& d : dyn_) ex.append(rows, d.row, d.len, sum_coef(s, column_value(d.col)), t);
        sym_merge(t);
        pb.combine(nf[s], t.data(), t.size(), len);
    }
    drop_fold(rows);
    for (unsigned s = 0; s < 3; ++s) fold_[s] = nf[s];
    fold_len_ = len;
    dyn_.clear();
    return true;
}

void LaneSums::drop_fold(RowTable& rows) {
    for (unsigned s = 0; s < 3; ++s) {
        rows.free_deferred(fold_[s]);
        fold_[s] = kNoRow;
    }
    fold_len_ = 0;
}

void LaneSums::read(RowTable& rows, const ExpansionTable& ex, Sym& out, const uint8_t* c, uint32_t limit,
                    ProgramBuilder* pb, bool short_scan) {
    if (!limit || (!c[0] && !c[1] && !c[2])) return;
    TAMD_PROF_SCOPE(kLaneRead);
    const uint32_t clip = content_ < limit ? content_ : limit;
    if (!terms_.empty()) {
        const uint32_t at = n_;
        RowId snap = kNoRow;
        for (size_t i = snaps_.size(); i-- > 0 && snaps_[i].after == at;)
            if (same_coefs(snaps_[i].c, c)) { snap = snaps_[i].row; break; }
        if (snap == kNoRow) {
            snap = rows.alloc(content_);
            if (snap == kNoRow) return;  // caller checks arena exhaustion via RowTable
            // written by the scan's chain (or only) op
            const uint32_t level = short_scan && at <= chunk() ? snap_level(rows, base_, 1) : snap_level(rows, base_);
            rows.set_level(snap, level);
            snaps_.push_back(Snap{snap, at, {c[0], c[1], c[2]}, (uint8_t)level});
        }
        if (clip) out.push_back(Term{snap, clip, 1});
    } else if (clip) {
        for (unsigned s = 0; s < 3; ++s)
            if (base_[s] != kNoRow && c[s]) out.push_back(Term{base_[s], clip, c[s]});
    }
    TAMD_PROF_SCOPE(kLaneDyn);
    const uint32_t fold_at = dyn_fold_above();
    // (only where expansions are limited -- the few-stream sessions and the C ABI, whose
    // decoders pile up recovered packets at high loss; the batched sessions inline everything
    // and a fold there costs a level for little: 1.05x the control time on the headline)
    if (pb && fold_at && dyn_.size() >= fold_at && ex.expand_limit != ~0u) fold_dyn(rows, *pb, ex);
    for (unsigned s = 0; s < 3; ++s)
        if (fold_[s] != kNoRow && c[s]) out.push_back(Term{fold_[s], fold_len_ < limit ? fold_len_ : limit, c[s]});
    for (const T& d : dyn_) {
        const uint32_t l = d.len < limit ? d.len : limit;
        const uint8_t cx = column_value(d.col);
        const uint8_t k = (uint8_t)(c[0] ^ gf_mul(c[1], cx) ^ gf_mul(c[2], gf_sqr(cx)));
        ex.append(rows, d.row, l, k, out);
    }
}

// Emit packets [from, to) of a run list; `ri`/`rdone` is a cursor (run index, packets of it done).
static void emit_packets(ProgramBuilder& pb, const std::vector<LaneSums::T>& terms, size_t& ri, uint32_t& rdone,
                         uint32_t count) {
    while (count > 0 && ri < terms.size()) {
        const LaneSums::T& t = terms[ri];
        uint32_t take = t.count - rdone;
        if (take > count) take = count;
        const uint32_t col = (t.col + kLanes * rdone) % TAMD_COLUMN_PERIOD;
        if (take == 1) {
            const uint8_t cx = column_value(col);
            pb.op_acc3_off(t.off + t.stride * rdone, cx, gf_sqr(cx), t.len);
        } else {
            pb.op_accr(TAMD_R_LANE3, 0, t.off + t.stride * rdone, t.stride, take, t.len, col, kLanes);
        }
        rdone += take;
        count -= take;
        if (rdone == t.count) {
            ++ri;
            rdone = 0;
        }
    }
}

// Advance a run-list cursor past `count` packets without emitting them.
static void skip_packets(const std::vector<LaneSums::T>& terms, size_t& ri, uint32_t& rdone, uint32_t count) {
    while (count > 0 && ri < terms.size()) {
        const uint32_t left = terms[ri].count - rdone;
        if (left > count) {
            rdone += count;
            return;
        }
        count -= left;
        ++ri;
        rdone = 0;
    }
}

uint32_t LaneSums::inline_max() {
    static const uint32_t v = getenv("TONK_AMD_INLINE_SEG") ? (uint32_t)atoi(getenv("TONK_AMD_INLINE_SEG")) : 3u;  // A/B
    return v;
}

// One scan = the lane's packets in order with snapshots (STOREC) at their read points.  A long
// scan would be one wave walking hundreds of rows, so it is cut into chunks of at most kChunk
// packets, split at every snapshot point: each chunk op (level 1) writes its three partial sums
// (deltas), and a chain op (level 2) adds base + deltas in order and takes the snapshots.
void LaneSums::emit_scan(RowTable& rows, ProgramBuilder& pb, const RowId* base, const std::vector<T>& terms,
                         const std::vector<Snap>& snaps, const RowId* final_rows) {
    static const uint8_t unit[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    uint32_t n = 0, width = 0;
    for (const T& t : terms) {
        n += t.count;
        if (t.len > width) width = t.len;
    }
    size_t si = 0, ri = 0;
    uint32_t rdone = 0;
    auto snapshots = [&](uint32_t pos) {
        while (si < snaps.size() && snaps[si].after == pos) {
            pb.op_storec(snaps[si].row, rows.cap_bytes(snaps[si].row), snaps[si].c);
            ++si;
        }
    };
    const uint32_t kChunk = chunk();
    // (a snapshot promised a lower level than the chain's -- LaneSums::read -- keeps the scan one op)
    const uint32_t chain_level = snap_level(rows, base);
    uint32_t level = chain_level;
    for (const Snap& sn : snaps)
        if (sn.level < level) level = sn.level;
    if (n <= kChunk || level < chain_level) {
        pb.begin_op();
        for (unsigned s = 0; s < 3; ++s)
            if (base[s] != kNoRow) pb.op_acc(base[s], 1, rows.cap_bytes(base[s]), s);
        uint32_t pos = 0;
        while (pos < n) {
            snapshots(pos);
            uint32_t until = si < snaps.size() ? snaps[si].after : n;
            if (until > n) until = n;
            emit_packets(pb, terms, ri, rdone, until - pos);
            pos = until;
        }
        snapshots(n);
        if (final_rows)
            for (unsigned s = 0; s < 3; ++s)
                if (final_rows[s] != kNoRow) pb.op_storec(final_rows[s], rows.cap_bytes(final_rows[s]), unit[s]);
        pb.end_op(level);
        return;
    }

    // Segments: cut at every snapshot point, and at most kChunk packets apart.  A segment of
    // more than inline_max() packets is a chunk op (level 1) whose three partial sums go to one
    // row of three parts; the chain op adds them.  A shorter one is walked by the chain op
    // itself: its packets are read once, where a chunk would write three partial rows and the
    // chain read them back (dense snapshots -- a recovery row every few lane packets -- made most
    // chunks one to three packets long).
    struct Seg { uint32_t pos, count; RowId delta; };
    thread_local std::vector<Seg> segs;
    segs.clear();
    const uint32_t wunits = (width + TAMD_ROW_UNIT - 1) / TAMD_ROW_UNIT;
    const uint32_t wcap = wunits * TAMD_ROW_UNIT;
    const uint32_t imax = inline_max();
    uint32_t pos = 0;
    size_t sj = 0;
    while (pos < n) {
        while (sj < snaps.size() && snaps[sj].after <= pos) ++sj;
        uint32_t end = pos + kChunk;
        if (sj < snaps.size() && snaps[sj].after < end) end = snaps[sj].after;
        if (end > n) end = n;
        Seg g{pos, end - pos, kNoRow};
        if (g.count <= imax) {
            skip_packets(terms, ri, rdone, g.count);
        } else {
            pb.begin_op();
            emit_packets(pb, terms, ri, rdone, g.count);
            g.delta = rows.alloc(3 * wcap);
            if (g.delta != kNoRow)
                for (unsigned s = 0; s < 3; ++s) pb.op_storec_part(g.delta, s * wunits, wcap, wcap, unit[s], s == 0);
            pb.end_op(1);
        }
        segs.push_back(g);
        pos = end;
    }
    ri = 0;
    rdone = 0;
    pb.begin_op();
    for (unsigned s = 0; s < 3; ++s)
        if (base[s] != kNoRow) pb.op_acc(base[s], 1, rows.cap_bytes(base[s]), s);
    for (const Seg& g : segs) {
        snapshots(g.pos);
        if (g.count <= imax) {
            emit_packets(pb, terms, ri, rdone, g.count);
        } else {
            skip_packets(terms, ri, rdone, g.count);
            if (g.delta != kNoRow)
                for (unsigned s = 0; s < 3; ++s) pb.op_acc_part(g.delta, s * wunits, 1, wcap, s);
        }
    }
    snapshots(n);
    if (final_rows)
        for (unsigned s = 0; s < 3; ++s)
            if (final_rows[s] != kNoRow) pb.op_storec(final_rows[s], rows.cap_bytes(final_rows[s]), unit[s]);
    pb.end_op(snap_level(rows, base));
    for (const Seg& g : segs) rows.free_deferred(g.delta);  // read only inside this program
}

void LaneSums::flush(RowTable& rows, ProgramBuilder& pb, const ExpansionTable& ex) {
    TAMD_PROF_SCOPE(kChainFlush);
    for (size_t i = 0; i < n_closed_; ++i) {
        Closed& c = closed_[i];
        emit_scan(rows, pb, c.base, c.terms, c.snaps, nullptr);
        for (unsigned s = 0; s < 3; ++s) rows.free_deferred(c.base[s]);
        for (const Snap& sn : c.snaps) rows.free_deferred(sn.row);
    }
    n_closed_ = 0;

    const bool folded = fold_[0] != kNoRow;
    if (terms_.empty() && dyn_.empty() && !folded) {
        // Nothing accumulated since the last flush: snapshots (if any) alias the bases.
        snaps_.clear();
        return;
    }

    RowId state[3] = {base_[0], base_[1], base_[2]};  // rows holding the static values after the scan
    bool state_is_new = false;
    if (!terms_.empty()) {
        RowId final_rows[3] = {kNoRow, kNoRow, kNoRow};
        for (unsigned s = 0; s < 3; ++s) {
            final_rows[s] = rows.alloc(content_);
            state[s] = final_rows[s];
        }
        emit_scan(rows, pb, base_, terms_, snaps_, final_rows);
        for (const Snap& sn : snaps_) rows.free_deferred(sn.row);
        state_is_new = true;
    }

    if (!dyn_.empty() || folded) {
        // Fold contributions of rows produced by this program into the carried values.
        for (unsigned s = 0; s < 3; ++s) {
            Sym t;
            if (state[s] != kNoRow) t.push_back(Term{state[s], rows.cap_bytes(state[s]), 1});
            if (fold_[s] != kNoRow) t.push_back(Term{fold_[s], fold_len_, 1});
            for (const T& d : dyn_) ex.append(rows, d.row, d.len, sum_coef(s, column_value(d.col)), t);
            sym_merge(t);
            const RowId carry = rows.alloc(content_);
            pb.combine(carry, t.data(), t.size(), content_);
            if (state_is_new) rows.free_deferred(state[s]);
            if (base_[s] != kNoRow) rows.free_deferred(base_[s]);
            base_[s] = carry;
        }
    } else {
        for (unsigned s = 0; s < 3; ++s) {
            if (base_[s] != kNoRow && base_[s] != state[s]) rows.free_deferred(base_[s]);
            base_[s] = state[s];
        }
    }
    terms_.clear();
    n_ = 0;
    snaps_.clear();
    dyn_.clear();
    drop_fold(rows);
}

void LaneSums::release(RowTable& rows) {
    for (size_t i = 0; i < n_closed_; ++i) {
        Closed& c = closed_[i];
        for (unsigned s = 0; s < 3; ++s) rows.free_deferred(c.base[s]);
        for (const Snap& sn : c.snaps) rows.free_deferred(sn.row);
    }
    n_closed_ = 0;
    for (const Snap& sn : snaps_) rows.free_deferred(sn.row);
    for (unsigned s = 0; s < 3; ++s) {
        rows.free_deferred(base_[s]);
        base_[s] = kNoRow;
    }
    terms_.clear();
    n_ = 0;
    snaps_.clear();
    dyn_.clear();
    drop_fold(rows);
    content_ = bytes = 0;
}

// ---------------------------------------------------------------------------------------------
RowId fold_low_levels(RowTable& rows, ProgramBuilder& pb, Sym& s, uint32_t keep_level,
                      uint32_t len, uint32_t row_bytes) {
    (void)row_bytes;
    thread_local Sym low, high;
    low.clear();
    high.clear();
    for (const Term& t : s) {
        if (is_run(t.row) || rows.level(t.row) < keep_level) low.push_back(t);
        else high.push_back(t);
    }
    sym_merge(low);
    if (low.empty()) { s.swap(high); return kNoRow; }
    if (low.size() == 1 && low[0].coef == 1) {
        high.push_back(low[0]);
        s.swap(high);
        return kNoRow;
    }
    const RowId r = rows.alloc(len);
    if (r == kNoRow) return kNoRow;
    pb.combine(r, low.data(), low.size(), len);
    high.push_back(Term{r, len, 1});
    s.swap(high);
    return r;
}

} // namespace tamd
