// decoder.cpp -- Siamese decoder control plane.  Each function names the reference routine it
// restates (SiameseDecoder.cpp line numbers); byte work becomes symbolic terms (engine.h).
#include "decoder.h"
#include "prof.h"

#include <algorithm>
#include <stdlib.h>
#include <string.h>

namespace tamd {

// Term lists up to this length go to the device unmerged (see eliminate_original_data).
static const size_t kMergeAbove = 48;

static inline uint32_t popcount64(uint64_t x) { return (uint32_t)__builtin_popcountll(x); }

// CustomBitSet<64> helpers (PacketAllocator.h:243-346)
static inline uint32_t bits_popcount(uint64_t w, uint32_t start, uint32_t end) {
    if (start >= end) return 0;
    const uint32_t n = end - start;
    const uint64_t mask = n >= 64 ? ~0ull : ((1ull << n) - 1);
    return popcount64((w >> start) & mask);
}
static inline uint32_t bits_first_clear(uint64_t w, uint32_t start) {
    const uint64_t v = (~w) >> start;
    if (start >= 64 || v == 0) return 64;
    return start + (uint32_t)__builtin_ctzll(v);
}
static inline uint32_t bits_first_set(uint64_t w, uint32_t start) {
    const uint64_t v = w >> start;
    if (start >= 64 || v == 0) return 64;
    return start + (uint32_t)__builtin_ctzll(v);
}

Decoder::Decoder(Context* ctx, uint32_t row_bytes, HostRelease release, void* user)
    : ctx_(ctx), row_bytes_(row_bytes), release_(release), user_(user) {
    ctx_->attach(this);
}

Decoder::~Decoder() {
    for (Subwindow* s : subs_) {
        for (unsigned i = 0; i < kSubwindow; ++i) drop_original(s->orig[i]);
        delete s;
    }
    subs_.clear();
    for (size_t i = 0; i < segs_.size(); ++i) release_segment(segs_[i], 0, segs_[i].count);
    segs_.clear();
    Recovery* r = head_;
    while (r) { Recovery* n = r->next; free_recovery(r); r = n; }
    for (Recovery* g : graveyard_) delete g;
    graveyard_.clear();
    for (Recovery* g : pool_) delete g;
    pool_.clear();
    pre_flush();  // snapshots already referenced by the pending program must still be written
    for (unsigned l = 0; l < kLanes; ++l) lanes_[l].sums.release(ctx_->rows);
    ctx_->detach(this);
}

void Decoder::pre_flush() {
    for (unsigned l = 0; l < kLanes; ++l) lanes_[l].sums.flush(ctx_->rows, ctx_->pb, ctx_->ex);
}

void Decoder::drop_original(StoredOriginal& o) {
    if (o.owned) ctx_->rows.free_deferred(o.row);
    if (o.host && release_) release_(o.host, user_);
    // an empty slot is bytes == 0, run == 0, owned == 0 and host == null (every add writes all
    // the other fields; a cleared subwindow is all zero)
    o.row = kNoRow;
    o.bytes = 0;
    o.owned = 0;
    o.host = nullptr;
    o.run = 0;
}

void Decoder::free_recovery(Recovery* r) {
    if (r->row != kNoRow) ctx_->rows.free_deferred(r->row);
    r->row = kNoRow;
    graveyard_.push_back(r);
}

void Decoder::read_original(RowId row, uint32_t len, uint8_t coef, Sym& out) const {
    ctx_->ex.append(ctx_->rows, row, len, coef, out);
}

void Decoder::release_segment(const Segment& s, uint32_t from, uint32_t n) {
    if (s.owned)
        for (uint32_t j = from; j < from + n; ++j) ctx_->rows.free_deferred(s.row(j));
}

void Decoder::append(uint32_t e0, const RowId* rows, uint32_t k, uint32_t framed_bytes, uint32_t header_bytes,
                     uint8_t owned, uint64_t layout) {
    const RowTable& rt = ctx_->rows;
    uint32_t e = e0, col = to_column(e0);
    // Fast path: the k packets are consecutive handles at one offset stride with no column wrap
    // inside (a stretch of a session's inputs): they continue the last segment or open one, and
    // only the elements' segment numbers are filled.
    if (k >= 2 && col + k - 1 < kColumnPeriod && col != 0 && (layout || consecutive_handles(rows, k))) {
        const uint32_t o0 = layout ? (uint32_t)(layout >> 32) : rt.offset(rows[0]);
        const uint32_t o1 = layout ? o0 + (uint32_t)layout : rt.offset(rows[1]);
        const uint32_t stride = o1 - o0;
        if (o1 > o0 && (layout || rt.affine(rows[0], k, stride))) {
            Segment* last = segs_.empty() ? nullptr : &segs_.back();
            const bool cont = last && last->end() == e0 + base_ && last->bytes == framed_bytes &&
                              last->header_bytes == header_bytes && last->owned == owned &&
                              rows[0] == last->row0 + last->count && o0 > last->off0 &&
                              (last->count == 1 ? o0 - last->off0 == stride
                                                : last->stride == stride && o0 == last->off(last->count));
            if (cont) {
                last->stride = stride;
                last->count += k;
            } else {
                Segment sg;
                sg.first = e0 + base_;
                sg.count = k;
                sg.row0 = rows[0];
                sg.off0 = o0;
                sg.stride = stride;
                sg.bytes = framed_bytes;
                sg.column0 = col;
                sg.header_bytes = (uint8_t)header_bytes;
                sg.owned = owned;
                segs_.push_back(sg);
            }
            const uint32_t id = seg_base_ + (uint32_t)segs_.size() - 1;
            for (uint32_t x = e0; x < e0 + k;) {
                const uint32_t bit = x % kSubwindow;
                const uint32_t n = std::min(kSubwindow - bit, e0 + k - x);
                std::fill_n(subs_[x / kSubwindow]->seg + bit, n, id);
                x += n;
            }
            return;
        }
    }
    uint32_t j = 0;
    while (j < k) {
        Segment* last = segs_.empty() ? nullptr : &segs_.back();
        const uint32_t e_abs = e + base_;
        const RowId r = rows[j];
        const uint32_t off = rt.offset(r);
        const bool cont = last && last->end() == e_abs && last->bytes == framed_bytes &&
                          last->header_bytes == header_bytes && last->owned == owned && r == last->row0 + last->count &&
                          off > last->off0 && col != 0 && (last->count == 1 || off == last->off(last->count));
        if (cont) {
            if (last->count == 1) last->stride = off - last->off0;
            ++last->count;
        } else {
            Segment sg;
            sg.first = e_abs;
            sg.count = 1;
            sg.row0 = r;
            sg.off0 = off;
            sg.bytes = framed_bytes;
            sg.column0 = col;
            sg.header_bytes = (uint8_t)header_bytes;
            sg.owned = owned;
            segs_.push_back(sg);
            last = &segs_.back();
        }
        const uint32_t id = seg_base_ + (uint32_t)segs_.size() - 1;
        subs_[e / kSubwindow]->seg[e % kSubwindow] = id;
        ++e;
        ++j;
        col = col_inc(col);
        // the rest of the run while rows keep both strides: only the element's segment number
        if (last->count >= 2) {
            uint32_t n = last->count;
            while (j < k && rows[j] == last->row0 + n && col != 0 && rt.offset(rows[j]) == last->off(n)) {
                subs_[e / kSubwindow]->seg[e % kSubwindow] = id;
                ++e;
                ++j;
                ++n;
                col = col_inc(col);
            }
            last->count = n;
        }
    }
}

// ============================================================================================
// Window (SiameseDecoder.cpp:1260-1536)
// ============================================================================================

// DecoderPacketWindow::MarkGotColumn (:1260-1277)
bool Decoder::mark_got(uint32_t column) {
    const uint32_t e = to_element(column);
    if (invalid_element(e)) { disabled_ = true; return false; }
    Subwindow* s = subs_[e / kSubwindow];
    s->got_count++;
    s->got |= 1ull << (e % kSubwindow);
    return e == next_expected_;
}

// RangeLostPackets (:1279-1323)
uint32_t Decoder::range_lost(uint32_t start, uint32_t end) {
    if (start >= end) return 0;
    uint32_t lost = 0;
    uint32_t sub = start / kSubwindow;
    const uint32_t bit = start % kSubwindow;
    if (bit > 0) {
        uint32_t bit_end = bit + end - start;
        if (bit_end > kSubwindow) bit_end = kSubwindow;
        lost += (bit_end - bit) - bits_popcount(subs_[sub]->got, bit, bit_end);
        ++sub;
    }
    const uint32_t sub_end = end / kSubwindow;
    for (uint32_t i = sub; i < sub_end; ++i) lost += kSubwindow - subs_[i]->got_count;
    if (sub_end >= sub) {
        const uint32_t last_bits = end - sub_end * kSubwindow;
        if (last_bits > 0) lost += last_bits - bits_popcount(subs_[sub_end]->got, 0, last_bits);
    }
    return lost;
}

// FindNextLostElement (:1325-1370)
uint32_t Decoder::find_next_lost(uint32_t start) {
    if (start >= count_) return count_;
    const uint32_t sub_end = (count_ + kSubwindow - 1) / kSubwindow;
    uint32_t sub = start / kSubwindow, bit = start % kSubwindow;
    while (sub < sub_end) {
        if (subs_[sub]->got_count < kSubwindow) {
            bit = bits_first_clear(subs_[sub]->got, bit);
            if (bit < kSubwindow) {
                uint32_t e = sub * kSubwindow + bit;
                if (e > count_) e = count_;
                return e;
            }
        }
        bit = 0;
        ++sub;
    }
    return count_;
}

// FindNextGotElement (:1372-1417)
uint32_t Decoder::find_next_got(uint32_t start) {
    if (start >= count_) return count_;
    const uint32_t sub_end = (count_ + kSubwindow - 1) / kSubwindow;
    uint32_t sub = start / kSubwindow, bit = start % kSubwindow;
    while (sub < sub_end) {
        if (subs_[sub]->got_count > 0) {
            bit = bits_first_set(subs_[sub]->got, bit);
            if (bit < kSubwindow) {
                uint32_t e = sub * kSubwindow + bit;
                if (e > count_) e = count_;
                return e;
            }
        }
        bit = 0;
        ++sub;
    }
    return count_;
}

// IterateNextExpectedElement (:1419-1434)
void Decoder::iterate_next_expected(uint32_t start) {
    if (next_expected_ >= count_) return;
    next_expected_ = find_next_lost(start);
}

// GrowWindow (:1436-1465)
bool Decoder::grow_window(uint32_t end) {
    const uint32_t needed = (end + kLanes + kSubwindow - 1) / kSubwindow;
    while (subs_.size() < needed) subs_.push_back(new Subwindow());
    if (end > count_) count_ = end;
    return true;
}

// DecoderPacketWindow::AddOriginal (:1467-1536)
Result Decoder::add_original(uint32_t packet_num, RowId row, uint32_t framed_bytes, uint32_t header_bytes,
                             uint32_t payload_bytes, void* host, bool* took, bool borrowed) {
    *took = false;
    if (disabled_) return kDisabled;
    const uint32_t e = to_element(packet_num);
    if (col_delta_negative(e)) {
        stats_[6]++;
        return kDuplicateData;
    }
    const bool at_end = e >= count_;  // (beyond every element so far: may continue a segment)
    grow_window(e + 1);
    Subwindow* s = subs_[e / kSubwindow];
    const uint32_t bit = e % kSubwindow;
    if ((s->got >> bit) & 1u) {
        stats_[6]++;
        return kDuplicateData;
    }
    if (at_end && !host) {
        append(e, &row, 1, framed_bytes, header_bytes, borrowed ? 0 : 1);
    } else {
        StoredOriginal& o = s->orig[bit];
        drop_original(o);
        o.row = row;
        o.off = ctx_->rows.offset(row);
        o.bytes = framed_bytes;
        o.column = packet_num;
        o.header_bytes = (uint8_t)header_bytes;
        o.owned = borrowed ? 0 : 1;
        o.host = host;
        o.run = 0;
        o.stride = 0;
        if (o.owned || host) s->held |= 1ull << bit;
        s->singles |= 1ull << bit;
    }
    *took = !borrowed;
    s->got_count++;
    s->got |= 1ull << bit;

    if (e == next_expected_) {
        iterate_next_expected(e + 1);
        list_delete_before(next_expected_);
    }
    if (e >= cr_.element_start && e < cr_.next_check_start) checked_reset();

    stats_[0]++;
    stats_[1] += payload_bytes;
    return kSuccess;
}

// k add_original() calls for the next columns col0 .. col0 + k - 1 (rows[0..k)), each followed
// by an is_ready() that fails, batched.  The new elements lie beyond the window end, so each call
// only stores the row, sets its got bit and moves NextExpected along (SiameseDecoder.cpp:
// 1467-1536 restated for that case); is_ready() cannot succeed when no recovery is pending.
bool Decoder::add_run_inorder(uint32_t col0, const RowId* rows, uint32_t k, uint32_t framed_bytes,
                              uint32_t header_bytes, uint32_t payload_bytes, bool borrowed, uint64_t layout) {
    if (disabled_ || has_recovered_ || !k) return false;
    const uint32_t e0 = to_element(col0);
    if (col_delta_negative(e0) || e0 < count_) return false;
    // Recovery packets pending: the run is still batchable when an earlier element is lost (so
    // NextExpected stays put and no recovery is deleted) and the decoder is not ready now.  The
    // new elements lie past every pending recovery's range, so each single call's is_ready()
    // would repeat this answer without changing any state.
    if (head_ && (next_expected_ >= e0 || check_recovery_possible())) return false;
    grow_window(e0 + k);
    append(e0, rows, k, framed_bytes, header_bytes, borrowed ? 0 : 1, layout);
    for (uint32_t e = e0; e < e0 + k;) {  // got bits a subwindow at a time
        const uint32_t bit = e % kSubwindow;
        const uint32_t n = std::min(kSubwindow - bit, e0 + k - e);
        Subwindow* s = subs_[e / kSubwindow];
        s->got |= (n == 64 ? ~0ull : ((1ull << n) - 1)) << bit;
        s->got_count += n;
        e += n;
    }
    if (e0 == next_expected_) next_expected_ = find_next_lost(e0 + k);
    if (std::max(e0, cr_.element_start) < std::min(e0 + k, cr_.next_check_start)) checked_reset();
    stats_[0] += k;
    stats_[1] += (uint64_t)payload_bytes * k;
    return true;
}

// PlugSumHoles (:1538-1602)
bool Decoder::plug_sum_holes(uint32_t element_start) {
    for (uint32_t column : recovered_columns_) {
        const uint32_t e = to_element(column);
        if (invalid_element(e)) continue;
        const uint32_t lane = column % kLanes;
        const uint32_t lane_start = next_lane_element(element_start, lane);
        LaneSum& sum = lanes_[lane];
        if (e >= lane_start && e < sum.element_end) {
            const StoredOriginal& o = elem(e);
            if (o.bytes <= 0) return false;
            sum.sums.grow(o.bytes);
            sum.sums.accumulate(ctx_->rows, o.row, o.bytes, column);
        }
    }
    recovered_columns_.clear();
    return true;
}

// ResetSums (:1604-1627)
void Decoder::reset_sums(uint32_t element_start) {
    for (unsigned l = 0; l < kLanes; ++l) {
        const uint32_t ls = next_lane_element(element_start, l);
        LaneSum& sum = lanes_[l];
        sum.element_start = ls;
        sum.element_end = ls;
        sum.sums.reset(ctx_->rows);
    }
    recovered_columns_.clear();
}

// StartSums (:1629-1678)
bool Decoder::start_sums(uint32_t element_start, uint32_t buffer_bytes) {
    for (unsigned l = 0; l < kLanes; ++l) {
        const uint32_t ls = next_lane_element(element_start, l);
        LaneSum& sum = lanes_[l];
        if (sum.sums.bytes == 0) {
            sum.element_end = ls;
        } else if (sum.element_start != ls) {
            sum.element_end = ls;
            sum.sums.reset(ctx_->rows);
        }
        sum.element_start = ls;
        sum.sums.grow(buffer_bytes);
    }
    if (!recovered_columns_.empty() && !plug_sum_holes(element_start)) return false;
    return true;
}

// DecoderPacketWindow::GetSum (:1680-1739), for the lane's three sums at once.  The lane's
// packets inside a segment are every kLanes-th of it: one strided run per segment.
LaneSums& Decoder::get_lane(uint32_t lane, uint32_t element_end) {
    LaneSum& sum = lanes_[lane];
    uint32_t e = sum.element_end;
    if (e >= element_end) return sum.sums;
    do {
        const uint32_t id = seg_id(e);
        if (id != kSingle) {
            const Segment& sg = segs_[id - seg_base_];
            const uint32_t j = e + base_ - sg.first;
            uint32_t stop = sg.end() - base_;
            if (stop > element_end) stop = element_end;
            const uint32_t n = (stop - 1 - e) / kLanes + 1;
            sum.sums.grow(sg.bytes);
            sum.sums.accumulate_run_level0(sg.row(j), sg.off(j), sg.bytes, col_add(sg.column0, j), n, sg.stride * kLanes);
            e += n * kLanes;
            continue;
        }
        const StoredOriginal& o = elem(e);
        if (o.bytes > 0) {
            sum.sums.grow(o.bytes);
            if (ctx_->rows.level(o.row) == 0) sum.sums.accumulate_level0(o.row, ctx_->rows.offset(o.row), o.bytes, o.column);
            else sum.sums.accumulate(ctx_->rows, o.row, o.bytes, o.column);
        }
        e += kLanes;
    } while (e < element_end);
    sum.element_end = e;
    return sum.sums;
}

// RemoveElements' walk over the recovery list (:1790-1830): the smallest element start, the
// largest packet, the first sum row, and the first sum elements of the other sum rows that differ
// from it (any of those outside the window disables the decoder).
void Decoder::list_walk(ListWalk& w) const {
    w.min_start = ~0u;
    w.max_bytes = 0;
    w.seen_sum = false;
    w.target_start = w.target_count = 0;
    w.min_fse = ~0u;
    w.invalid = false;
    for (const Recovery* r = head_; r; r = r->next) {
        const uint32_t sc = r->meta.SumCount, cs = r->meta.ColumnStart;
        if (sc > kCauchyThreshold) {
            if (!w.seen_sum) {
                w.target_start = cs;
                w.target_count = sc;
                w.target_end = r->element_end;
                w.seen_sum = true;
            } else if (cs != w.target_start || sc < w.target_count) {
                const uint32_t fse = to_element(cs);
                if (invalid_element(fse)) {
                    w.invalid = true;
                    return;
                }
                if (w.min_fse > fse) w.min_fse = fse;
            }
        }
        if (w.min_start > r->element_start) w.min_start = r->element_start;
        if (w.max_bytes < r->bytes) w.max_bytes = r->bytes;
    }
}

// DecoderPacketWindow::RemoveElements (:1778-2033)
void Decoder::remove_elements() {
    if (next_expected_ < kRemoveThreshold) return;

    uint32_t first_kept = 0, target_start = 0, target_count = 0, initial_bytes = 0;
    bool seen_sum = false;
    const Recovery* r = head_;
    if (!r) {
        const RecoveryMeta m = last_meta_;
        const uint32_t end = to_element(m.ColumnStart + m.SumCount);
        if (col_delta_negative(end) || end < m.LDPCCount) { disabled_ = true; return; }
        first_kept = end - m.LDPCCount;
        target_start = m.ColumnStart;
        target_count = m.SumCount;
        initial_bytes = last_bytes_;
        if (m.SumCount > kCauchyThreshold) seen_sum = true;
    } else {
        // (the walk below, or what it found last time when neither the list nor the window moved:
        // a decoder far behind holds thousands of recovery packets and calls this on every add)
        if (!(walk_.valid && walk_.gen == list_gen_ && walk_.column_start == column_start_ && walk_.count == count_)) {
            list_walk(walk_);
            walk_.valid = true;
            walk_.gen = list_gen_;
            walk_.column_start = column_start_;
            walk_.count = count_;
        }
        if (walk_.invalid) { disabled_ = true; return; }
        first_kept = walk_.min_start < walk_.min_fse ? walk_.min_start : walk_.min_fse;
        initial_bytes = walk_.max_bytes;
        seen_sum = walk_.seen_sum;
        target_start = walk_.target_start;
        target_count = walk_.target_count;
    }
    if (first_kept < kRemoveThreshold) return;

    const uint32_t first_kept_sub = first_kept / kSubwindow;
    const uint32_t removed = first_kept_sub * kSubwindow;

    if (seen_sum) {
        uint32_t sum_elem = to_element(target_start);
        if (sum_column_start_ != target_start || sum_column_count_ > target_count) {
            if (invalid_element(sum_elem)) { disabled_ = true; return; }
            reset_sums(sum_elem);
            sum_column_start_ = target_start;
            sum_column_count_ = target_count;
        } else {
            if (invalid_element(sum_elem)) sum_elem = 0;
            if (!start_sums(sum_elem, initial_bytes)) { disabled_ = true; return; }
        }
        for (unsigned l = 0; l < kLanes; ++l) {
            get_lane(l, removed);
            LaneSum& sum = lanes_[l];
            if (sum.element_start >= removed) sum.element_start -= removed;
            else sum.element_start = l;
            sum.element_end -= removed;
        }
    } else {
        sum_column_count_ = 0;
    }

    for (uint32_t i = 0; i < first_kept_sub; ++i) {
        Subwindow* s = subs_[i];
        // only the slots written since the last clear: those holding a row or host copy release
        // it, every one is zeroed (borrowed rows need no release)
        for (uint64_t m = s->held; m; m &= m - 1) drop_original(s->orig[__builtin_ctzll(m)]);
        for (uint64_t m = s->singles | s->held; m; m &= m - 1)
            memset((void*)&s->orig[__builtin_ctzll(m)], 0, sizeof(StoredOriginal));
        memset(s->seg, 0xff, sizeof(s->seg));
        s->got = 0;
        s->got_count = 0;
        s->held = 0;
        s->singles = 0;
    }
    std::rotate(subs_.begin(), subs_.begin() + first_kept_sub, subs_.end());
    // segments below the new window start leave; one that straddles it keeps its later packets
    const uint32_t cut = base_ + removed;
    while (!segs_.empty() && segs_.front().end() <= cut) {
        release_segment(segs_.front(), 0, segs_.front().count);
        segs_.pop_front(1);
        ++seg_base_;
    }
    if (!segs_.empty() && segs_.front().first < cut) {
        Segment& f = segs_.front();
        const uint32_t d = cut - f.first;
        release_segment(f, 0, d);
        f.first = cut;
        f.count -= d;
        f.row0 += d;
        f.off0 += d * f.stride;
        f.column0 = col_add(f.column0, d);
    }
    base_ = cut;

    count_ -= removed;
    column_start_ = to_column(removed);
    next_expected_ -= removed;

    ++list_gen_;
    for (Recovery* q = head_; q; q = q->next) {
        q->element_end -= removed;
        q->element_start -= removed;
    }
    checked_decrement(removed);
    prev_next_check_start_ = prev_next_check_start_ > removed ? prev_next_check_start_ - removed : 0;
}

// ============================================================================================
// Recovery list and checked region (:2537-2666)
// ============================================================================================

// RecoveryPacketList::Insert (:2567-2635)
void Decoder::list_insert(Recovery* rec, bool out_of_order) {
    Recovery* prev = tail_;
    Recovery* next = nullptr;
    const uint32_t rs = rec->meta.ColumnStart, re = rec->element_end;
    if (ins_gen_ == list_gen_ && ins_end_ == re && ins_start_ == rs) {
        // The walk from the tail passes every node it passed for the previous insertion, and that
        // node too (an equal key continues the walk), and stops where that walk stopped: the
        // packet goes right in front of it.  (The flush of a decoder far behind adds thousands of
        // recovery packets with one key, each walk ~2,000 nodes long.)
        next = ins_last_;
        prev = ins_last_->prev;
    } else {
        for (; prev; next = prev, prev = prev->prev) {
            const uint32_t ps = prev->meta.ColumnStart, pe = prev->element_end;
            if (re >= pe) {
                if (re > pe) break;
                if (col_delta_negative(col_sub(rs, ps))) break;
            }
        }
    }
    // remove_elements' walk over the list stays what it was, plus this packet, unless the packet
    // can become the sum target in front of the current one: a sum row is the target when it is
    // the first; one ending after the target's end goes behind it (the list is ordered by end)
    // and counts its first sum element if it differs from the target; one with the target's start
    // and count changes nothing wherever it goes.  Otherwise the next removal walks again.
    const uint32_t sc = rec->meta.SumCount;
    const bool is_sum = sc > kCauchyThreshold;
    const bool same_target = is_sum && walk_.seen_sum && rs == walk_.target_start && sc == walk_.target_count;
    const bool walk_kept = walk_.valid && walk_.gen == list_gen_ && walk_.column_start == column_start_ &&
                           walk_.count == count_ &&
                           (!is_sum || !walk_.seen_sum || same_target || re > walk_.target_end);
    ins_last_ = rec;
    ins_end_ = re;
    ins_start_ = rs;
    ins_gen_ = ++list_gen_;
    if (walk_kept) {
        if (is_sum && !walk_.seen_sum) {
            walk_.seen_sum = true;
            walk_.target_start = rs;
            walk_.target_count = sc;
            walk_.target_end = re;
        } else if (is_sum && !same_target && (rs != walk_.target_start || sc < walk_.target_count)) {
            const uint32_t fse = to_element(rs);
            if (invalid_element(fse)) walk_.invalid = true;
            else if (walk_.min_fse > fse) walk_.min_fse = fse;
        }
        if (walk_.min_start > rec->element_start) walk_.min_start = rec->element_start;
        if (walk_.max_bytes < rec->bytes) walk_.max_bytes = rec->bytes;
        walk_.gen = list_gen_;
    }
    rec->next = next;
    rec->prev = prev;
    if (prev) prev->next = rec; else head_ = rec;
    if (next) next->prev = rec; else tail_ = rec;
    if (!prev || next) checked_reset();
    ++recovery_count_;
    if (!out_of_order) {
        last_meta_ = rec->meta;
        last_bytes_ = rec->bytes;
    }
}

// RecoveryPacketList::DeletePacketsBefore (:2637-2666)
void Decoder::lazy_write() {
    Recovery* r = lazy_from_;
    for (uint32_t i = 0; i < lazy_n_ && r; ++i, r = r->next) r->lost_count = lazy_lost_;
    lazy_n_ = 0;
    lazy_from_ = nullptr;
}

void Decoder::list_delete_before(uint32_t element) {
    if (lazy_n_) lazy_write();
    ++list_gen_;
    Recovery* r = head_;
    uint32_t deleted = 0;
    while (r) {
        if (r->element_end > element) break;
        Recovery* n = r->next;
        free_recovery(r);
        ++deleted;
        r = n;
    }
    head_ = r;
    if (r) {
        r->prev = nullptr;
        recovery_count_ -= deleted;
    } else {
        tail_ = nullptr;
        recovery_count_ = 0;
    }
}

// CheckedRegionState::Reset (:2537-2548)
void Decoder::checked_reset() {
    cr_ = Checked();
    lazy_n_ = 0;  // (every loss count is written again before it is read)
    lazy_from_ = nullptr;
    matrix_reset();
    for (Recovery* r : graveyard_) pool_.push_back(r);  // reused by add_recovery
    graveyard_.clear();
}

// CheckedRegionState::DecrementElementCounters (:2550-2561)
void Decoder::checked_decrement(uint32_t n) {
    if (cr_.element_start < n || cr_.next_check_start < n) {
        checked_reset();
        return;
    }
    cr_.element_start -= n;
    cr_.next_check_start -= n;
}

// ============================================================================================
// Recovery matrix (:2039-2531)
// ============================================================================================

// RecoveryMatrixState::Reset (:2039-2049)
void Decoder::matrix_reset() {
    mcols_.clear();
    mrows_.clear();
    pivots_.clear();
    mat_rows_ = mat_cols_ = 0;
    prev_next_check_start_ = 0;
    ge_resume_pivot_ = 0;
}

// GrowingAlignedByteMatrix::Initialize / Resize (SiameseCommon.cpp:51-117).  Elements of the
// old matrix keep their values; the rest are written by generate_matrix before use.
bool Decoder::matrix_resize(uint32_t rows, uint32_t cols, bool keep) {
    if (keep && rows <= mat_alloc_rows_ && cols <= mat_stride_) {
        mat_rows_ = rows;
        mat_cols_ = cols;
        return true;
    }
    const uint32_t arows = rows + 4;
    const uint32_t acols = (cols + 4 + 31) & ~31u;
    std::vector<uint8_t> m((size_t)arows * acols, 0);
    if (keep && mat_cols_ > 0) {
        const uint32_t copy = mat_cols_ < cols ? mat_cols_ : cols;
        for (uint32_t i = 0; i < mat_rows_; ++i)
            memcpy(&m[(size_t)i * acols], &mat_[(size_t)i * mat_stride_], copy);
    }
    mat_.swap(m);
    mat_alloc_rows_ = arows;
    mat_stride_ = acols;
    mat_rows_ = rows;
    mat_cols_ = cols;
    return true;
}

// RecoveryMatrixState::PopulateColumns (:2059-2130)
void Decoder::populate_columns(uint32_t old_cols, uint32_t new_cols) {
    if (old_cols >= new_cols) return;
    mcols_.resize(new_cols);
    uint32_t start = prev_next_check_start_;
    prev_next_check_start_ = cr_.next_check_start;
    const uint32_t end = cr_.next_check_start;
    if (start < cr_.element_start) start = cr_.element_start;
    const uint32_t sub_end = (end + kSubwindow - 1) / kSubwindow;
    uint32_t sub = start / kSubwindow, bit = start % kSubwindow, column = old_cols;
    while (sub < sub_end) {
        Subwindow* s = subs_[sub];
        if (s->got_count < kSubwindow) {
            do {
                bit = bits_first_clear(s->got, bit);
                if (bit >= kSubwindow) break;
                const uint32_t e = sub * kSubwindow + bit;
                MatCol& c = mcols_[column];
                c.column = to_column(e);
                c.orig = &s->orig[bit];
                c.cx = column_value(c.column);
                c.orig->column = column;  // lost slot remembers its matrix column
                s->singles |= 1ull << bit;
                if (++column >= new_cols) return;
            } while (++bit < kSubwindow);
        }
        bit = 0;
        ++sub;
    }
    disabled_ = true;  // should never get here
}

// RecoveryMatrixState::PopulateRows (:2132-2155)
void Decoder::populate_rows(uint32_t old_rows, uint32_t new_rows) {
    if (old_rows >= new_rows) return;
    mrows_.resize(new_rows);
    Recovery* r = old_rows > 0 ? mrows_[old_rows - 1].rec->next : cr_.first;
    for (uint32_t i = old_rows; i < new_rows; ++i, r = r->next) {
        mrows_[i].rec = r;
        mrows_[i].used = false;
        mrows_[i].mcols = r->lost_count;
    }
}

// RecoveryMatrixState::GenerateMatrix (:2157-2383)
bool Decoder::generate_matrix() {
    if (lazy_n_) lazy_write();
    const uint32_t columns = cr_.lost_count;
    const uint32_t rows = cr_.recovery_count;
    uint32_t old_rows = (uint32_t)mrows_.size();
    uint32_t old_cols = (uint32_t)mcols_.size();
    if (rows < old_rows || columns < old_cols) {
        matrix_reset();
        old_rows = old_cols = 0;
    }
    matrix_resize(rows, columns, old_rows != 0);
    populate_columns(old_cols, columns);
    populate_rows(old_rows, rows);
    if (disabled_) return false;

    const uint32_t start_row = columns <= old_cols ? old_rows : 0;
    for (uint32_t i = start_row; i < rows; ++i) {
        Recovery* rec = mrows_[i].rec;
        const RecoveryMeta m = rec->meta;
        const uint32_t start_col = i < old_rows ? old_cols : 0;
        if (m.SumCount <= kCauchyThreshold) {
            for (uint32_t j = start_col; j < columns; ++j) {
                const uint32_t column = mcols_[j].column;
                const uint32_t e = col_sub(column, m.ColumnStart);
                if (e >= m.SumCount) {
                    for (; j < columns; ++j) mat(i, j) = 0;
                    break;
                }
                mat(i, j) = m.Row == 0 ? 1 : cauchy_element(m.Row - 1, column % kCauchyMaxColumns);
            }
            continue;
        }
        const uint8_t rx = row_value(m.Row);
        for (uint32_t j = start_col; j < columns; ++j) {
            const uint32_t column = mcols_[j].column;
            const uint32_t e = col_sub(column, m.ColumnStart);
            if (e >= m.SumCount) {
                for (; j < columns; ++j) mat(i, j) = 0;
                break;
            }
            const uint8_t cx = mcols_[j].cx, cx2 = gf_sqr(cx);
            const unsigned op = row_opcode(column % kLanes, m.Row);
            uint8_t v = 0;
            if (op & 1) v ^= 1;
            if (op & 2) v ^= cx;
            if (op & 4) v ^= cx2;
            if (op & 8) v ^= rx;
            if (op & 16) v ^= gf_mul(cx, rx);
            if (op & 32) v ^= gf_mul(cx2, rx);
            mat(i, j) = v;
        }
        Pcg32 prng;
        prng.seed(m.Row, m.LDPCCount);
        const uint32_t es = rec->element_start;
        const uint32_t pairs = (m.LDPCCount + kPairRate - 1) / kPairRate;
        const FastMod ldpc_mod(m.LDPCCount);
        for (uint32_t k = 0; k < pairs; ++k) {
            const uint32_t e1 = es + ldpc_mod(prng.next());
            if (!got(e1)) {  // a lost element: its slot holds its matrix column (populate_columns)
                const uint32_t mc = elem(e1).column;
                if (mc >= columns) { disabled_ = true; return false; }
                if (mc >= start_col) mat(i, mc) ^= 1;
            }
            const uint32_t erx = es + ldpc_mod(prng.next());
            if (!got(erx)) {
                const uint32_t mc = elem(erx).column;
                if (mc >= columns) { disabled_ = true; return false; }
                if (mc >= start_col) mat(i, mc) ^= rx;
            }
        }
    }
    pivots_.resize(rows);
    for (uint32_t i = old_rows; i < rows; ++i) pivots_[i] = i;
    if (ge_resume_pivot_ > 0) resume_ge(old_rows, rows);
    return true;
}

// RecoveryMatrixState::EliminateRow / MulAddRows (SiameseDecoder.h:504-541)
bool Decoder::eliminate_row(uint32_t ge_row, uint32_t rem_row, uint32_t pivot_i, uint32_t column_end, uint8_t val_i) {
    uint8_t* rem = &mat_[(size_t)rem_row * mat_stride_];
    const uint8_t* ge = &mat_[(size_t)ge_row * mat_stride_];
    const uint8_t val_j = rem[pivot_i];
    if (val_j == 0) return false;
    const uint8_t y = gf_div(val_j, val_i);
    rem[pivot_i] = y;
    const uint8_t* ymul = g_gf.mul[y];
    for (uint32_t c = pivot_i + 1; c < column_end; ++c) rem[c] ^= ymul[ge[c]];
    return true;
}

// RecoveryMatrixState::ResumeGE (:2385-2421)
void Decoder::resume_ge(uint32_t old_rows, uint32_t rows) {
    if (old_rows >= rows) return;
    for (uint32_t pi = 0; pi < ge_resume_pivot_; ++pi) {
        const uint32_t ri = pivots_[pi];
        const uint8_t val_i = mat(ri, pi);
        const uint32_t pcc = mrows_[ri].mcols;
        for (uint32_t nr = old_rows; nr < rows; ++nr) {
            if (eliminate_row(ri, nr, pi, pcc, val_i)) {
                if (mrows_[nr].mcols < pcc) mrows_[nr].mcols = pcc;
            }
        }
    }
}

// RecoveryMatrixState::GaussianElimination (:2423-2465)
bool Decoder::gaussian_elimination() {
    if (ge_resume_pivot_ > 0) return pivoted_ge(ge_resume_pivot_);
    const uint32_t columns = mat_cols_, rows = mat_rows_;
    for (uint32_t pi = 0; pi < columns; ++pi) {
        const uint8_t val_i = mat(pi, pi);
        if (val_i == 0) return pivoted_ge(pi);
        mrows_[pi].used = true;
        const uint32_t pcc = mrows_[pi].mcols;
        for (uint32_t pj = pi + 1; pj < rows; ++pj) eliminate_row(pi, pj, pi, pcc, val_i);
    }
    return true;
}

// RecoveryMatrixState::PivotedGaussianElimination (:2467-2531)
bool Decoder::pivoted_ge(uint32_t pivot_i) {
    const uint32_t columns = mat_cols_, rows = mat_rows_;
    uint32_t pj = pivot_i + 1;
    bool resume = true;
    for (; pivot_i < columns; ++pivot_i) {
        if (!resume) pj = pivot_i;
        resume = false;
        bool found = false;
        for (; pj < rows; ++pj) {
            const uint32_t rj = pivots_[pj];
            const uint8_t val_i = mat(rj, pivot_i);
            if (val_i == 0) continue;
            if (pivot_i != pj) std::swap(pivots_[pivot_i], pivots_[pj]);
            mrows_[rj].used = true;
            const uint32_t pcc = mrows_[rj].mcols;
            if (pivot_i >= columns - 1) return true;
            for (uint32_t pk = pivot_i + 1; pk < rows; ++pk) {
                const uint32_t rk = pivots_[pk];
                if (eliminate_row(rj, rk, pivot_i, pcc, val_i)) {
                    if (mrows_[rk].mcols < pcc) mrows_[rk].mcols = pcc;
                }
            }
            found = true;
            break;
        }
        if (!found) {
            ge_resume_pivot_ = pivot_i;
            return false;
        }
    }
    return true;
}

// ============================================================================================
// Decoder (SiameseDecoder.cpp:71-811)
// ============================================================================================

// Decoder::AddRecovery (:257-451)
Result Decoder::add_recovery(RowId row, uint32_t total_bytes, const uint8_t* tail, const uint8_t* host,
                             bool* took) {
    *took = false;
    if (disabled_) return kDisabled;
    RecoveryMeta m;
    const uint32_t tl = total_bytes < 8 ? total_bytes : 8;
    const int footer = get_recovery_footer(tail, tl, m);
    if (footer < 0) { disabled_ = true; return kDisabled; }

    stats_[2]++;
    stats_[3] += total_bytes;

    const bool out_of_order = col_delta_negative(m.ColumnStart + m.SumCount - latest_column_);
    if (!out_of_order) latest_column_ = (m.ColumnStart + m.SumCount) % kColumnPeriod;

    uint32_t es, ee;
    if (count_ <= 0) {
        if (out_of_order) { stats_[9]++; return kSuccess; }
        column_start_ = m.ColumnStart;
        grow_window(m.SumCount);
        ee = m.SumCount;
        es = ee - m.LDPCCount;
    } else {
        ee = to_element(m.ColumnStart + m.SumCount);
        if (col_delta_negative(ee)) { stats_[9]++; return kSuccess; }
        if (ee < m.LDPCCount) { stats_[9]++; return kSuccess; }
        es = ee - m.LDPCCount;
        if (ee <= next_expected_) {
            if (out_of_order) { stats_[9]++; return kSuccess; }
            if (es >= kRemoveThreshold) {
                last_meta_ = m;
                last_bytes_ = total_bytes - (uint32_t)footer;
                remove_elements();
            }
            stats_[9]++;
            return kSuccess;
        }
        if (m.SumCount > kCauchyThreshold) {
            if (sum_column_count_ == 0 || sum_column_start_ != m.ColumnStart) {
                if (invalid_element(to_element(m.ColumnStart))) { stats_[9]++; return kSuccess; }
            }
        }
        grow_window(ee);
    }

    if (m.SumCount == 1) {
        if (!add_single_recovery(row, total_bytes - (uint32_t)footer, host, m, took)) {
            disabled_ = true;
            return kDisabled;
        }
        return kSuccess;
    }

    Recovery* r;
    if (!pool_.empty()) {
        r = pool_.back();
        pool_.pop_back();
        r->next = r->prev = nullptr;
        r->lost_count = 0;
        r->buf.clear();
    } else {
        r = new Recovery();
    }
    r->bytes = total_bytes - (uint32_t)footer;
    r->row = row;
    *took = true;
    r->buf.push_back(Term{row, r->bytes, 1});
    r->meta = m;
    r->element_start = es;
    r->element_end = ee;
    list_insert(r, out_of_order);
    if (es >= kRemoveThreshold) remove_elements();
    return kSuccess;
}

// Decoder::AddSingleRecovery (:453-539).  The packet data is the framed original itself, so
// the window slot takes the packet row (its first `data_bytes` bytes) without a copy.
bool Decoder::add_single_recovery(RowId row, uint32_t data_bytes, const uint8_t* host,
                                  const RecoveryMeta& m, bool* took) {
    const uint32_t e = to_element(m.ColumnStart);
    if (invalid_element(e)) return false;
    if (got(e)) return true;
    StoredOriginal& o = elem(e);

    uint32_t header = 0, payload = 0;
    if (host) {
        unsigned len = 0;
        const int hb = get_length_header(host, data_bytes, len);
        if (hb < 1 || len == 0 || len + (unsigned)hb != data_bytes) return false;
        header = (uint32_t)hb;
        payload = len;
    }
    drop_original(o);
    o.row = row;
    o.off = ctx_->rows.offset(row);
    o.bytes = data_bytes;
    o.column = m.ColumnStart;
    o.header_bytes = (uint8_t)header;
    o.owned = 1;
    o.run = 0;
    o.stride = 0;
    subs_[e / kSubwindow]->held |= 1ull << (e % kSubwindow);
    subs_[e / kSubwindow]->singles |= 1ull << (e % kSubwindow);
    *took = true;

    if (!has_recovered_) {
        has_recovered_ = true;
        recovered_.clear();
    }
    RecoveredPacket rp;
    rp.packet_num = m.ColumnStart;
    rp.row = row;
    rp.framed_upper = data_bytes;
    rp.header_bytes = header;
    rp.data_bytes = payload;
    recovered_.push_back(rp);
    recovered_columns_.push_back(m.ColumnStart);

    if (e >= cr_.element_start && e < cr_.next_check_start) checked_reset();

    if (mark_got(m.ColumnStart)) {
        iterate_next_expected(e + 1);
        list_delete_before(next_expected_);
        if (cr_.next_check_start >= kRemoveThreshold) remove_elements();
    }
    return true;
}

// Decoder::CheckRecoveryPossible (:541-628)
bool Decoder::check_recovery_possible() {
    if (disabled_) return false;
    Recovery* r;
    uint32_t next_check, rcount, lost;
    if (!cr_.last) {
        r = head_;
        if (!r) return false;
        cr_.first = r;
        cr_.element_start = r->element_start;
        rcount = 1;
        next_check = r->element_end;
        lost = range_lost(r->element_start, next_check);
        cr_.solve_failed = false;
        r->lost_count = lost;
    } else {
        rcount = cr_.recovery_count;
        lost = cr_.lost_count;
        if (rcount >= lost && !cr_.solve_failed) return lost <= kMaxLossRecovery;
        r = cr_.last;
        next_check = cr_.next_check_start;
    }
    while ((rcount < lost || cr_.solve_failed) && r->next) {
        r = r->next;
        ++rcount;
        uint32_t ee = r->element_end;
        if (ee < next_check) ee = next_check;
        lost += range_lost(next_check, ee);
        next_check = ee;
        r->lost_count = lost;
        cr_.solve_failed = false;
    }
    cr_.last = r;
    cr_.recovery_count = rcount;
    cr_.lost_count = lost;
    cr_.next_check_start = next_check;
    if (lost > kMaxLossRecovery) return false;
    return rcount >= lost && !cr_.solve_failed;
}

Result Decoder::is_ready() {
    if (has_recovered_ || check_recovery_possible()) return kSuccess;
    return kNeedMoreData;
}

// Decoder::Decode (:630-727)
Result Decoder::decode(std::vector<RecoveredPacket*>& out) {
    if (disabled_) return kDisabled;
    if (has_recovered_) {
        has_recovered_ = false;
        for (RecoveredPacket& p : recovered_) out.push_back(&p);
        return kSuccess;
    }
    if (!check_recovery_possible()) return kNeedMoreData;

    Recovery* r = cr_.last;
    uint32_t next_check = cr_.next_check_start, rcount = cr_.recovery_count, lost = cr_.lost_count;
    // The checked region (cr_) only moves after this loop, so every attempt after a failed one
    // solves the same matrix again (GenerateMatrix reads CheckedRegion's counts, :2157-2165; the
    // resumed elimination stops at the same pivot without changing anything) and fails the same
    // way: those attempts are only counted (SolveFailCount), not repeated.  (A decoder far behind
    // -- stream 56 of configs[2] -- walks ~2,000 recovery packets per call, each an attempt.)
    bool failed = false;
    for (;;) {
        if (rcount >= lost) {
            if (failed) {
                stats_[8]++;
            } else {
                const Result res = decode_checked_region();
                if (res == kSuccess) {
                    for (RecoveredPacket& p : recovered_) out.push_back(&p);
                    return kSuccess;
                }
                if (res != kNeedMoreData) return res;
                failed = true;
            }
        }
        if (!r->next) break;
        if (failed && cr_.first == head_ && tail_->element_end <= next_check && !lazy_n_) {
            // The rest of the walk after a failed solve, at once: the list is ordered by element
            // end, so no later packet adds losses (its end is within next_check); each one counts
            // a failed attempt and faces `lost` losses.  r is the rcount-th packet from the head.
            const uint32_t rest = recovery_count_ - rcount;
            stats_[8] += rest;
            lazy_from_ = r->next;
            lazy_n_ = rest;
            lazy_lost_ = lost;
            rcount += rest;
            r = tail_;
            break;
        }
        r = r->next;
        ++rcount;
        uint32_t ee = r->element_end;
        if (ee < next_check) ee = next_check;
        lost += range_lost(next_check, ee);
        r->lost_count = lost;
        next_check = ee;
    }
    cr_.last = r;
    cr_.next_check_start = next_check;
    cr_.recovery_count = rcount;
    cr_.lost_count = lost;
    return kNeedMoreData;
}

// Decoder::DecodeCheckedRegion (:729-810)
Result Decoder::decode_checked_region() {
    {
        TAMD_PROF_SCOPE(kGenMatrix);
        if (!generate_matrix()) { disabled_ = true; return kDisabled; }
    }
    bool solved;
    {
        TAMD_PROF_SCOPE(kGE);
        solved = gaussian_elimination();
    }
    if (!solved) {
        cr_.solve_failed = true;
        stats_[8]++;
        return kNeedMoreData;
    }
    {
        TAMD_PROF_SCOPE(kElim);
        if (!eliminate_original_data()) { disabled_ = true; return kDisabled; }
    }
    {
        TAMD_PROF_SCOPE(kLowerTri);
        if (!multiply_lower_triangle()) { disabled_ = true; return kDisabled; }
    }
    Result res;
    {
        TAMD_PROF_SCOPE(kBackSub);
        res = back_substitution();
    }
    checked_reset();
    return res;
}

// Decoder::EliminateOriginalData (:812-1063)
bool Decoder::eliminate_original_data() {
    const uint32_t rows = cr_.recovery_count;
    for (uint32_t ri = 0; ri < rows; ++ri) {
        if (!mrows_[ri].used) continue;
        Recovery* rec = mrows_[ri].rec;
        const RecoveryMeta m = rec->meta;
        const uint32_t es = rec->element_start, ee = rec->element_end;
        Sym& buf = rec->buf;

        if (m.SumCount <= kCauchyThreshold) {
            // Received originals inside a segment (a run of equally long level-0 packets at one
            // row stride) enter as one run term: one ACCR run on the device, one term here.
            const uint32_t mode = m.Row == 0 ? TAMD_R_CONST : TAMD_R_CAUCHY;
            const uint32_t param = m.Row == 0 ? 1u : m.Row - 1;
            for (uint32_t j = es; j < ee; ++j) {
                const uint32_t id = seg_id(j);
                if (id != kSingle) {
                    const Segment& sg = segs_[id - seg_base_];
                    const uint32_t k = j + base_ - sg.first;
                    const uint32_t n = std::min(sg.end() - base_, ee) - j;
                    if (n >= 2) {
                        const uint32_t add = std::min(sg.bytes, rec->bytes);
                        buf.push_back(ctx_->pb.run_term(mode, param, sg.off(k), sg.stride, n, to_column(j), add));
                        j += n - 1;
                        continue;
                    }
                }
                RowId row;
                uint32_t add;
                if (!packet(j, row, add)) continue;
                if (add > rec->bytes) add = rec->bytes;
                const uint8_t y = m.Row == 0 ? 1 : cauchy_element(m.Row - 1, to_column(j) % kCauchyMaxColumns);
                read_original(row, add, y, buf);
            }
        } else {
            const uint32_t rbytes = rec->bytes;
            uint32_t sum_elem = to_element(m.ColumnStart);
            // (the sums' start is still in the window: no packet they would hold has been removed)
            const bool sum_valid = !invalid_element(sum_elem);
            {
            TAMD_PROF_SCOPE(kElimStart);
            if (m.ColumnStart != sum_column_start_ || m.SumCount < sum_column_count_) {
                if (invalid_element(sum_elem)) return false;
                reset_sums(sum_elem);
                sum_column_start_ = m.ColumnStart;
            } else {
                if (invalid_element(sum_elem)) sum_elem = 0;
                if (!start_sums(sum_elem, rbytes)) return false;
            }
            }
            sum_column_count_ = m.SumCount;
            if (sum_valid && ctx_->direct_elim && eliminate_direct(rec, sum_elem, buf)) {
                if (ctx_->oom) return false;
                if (cr_.lost_count == 1) {
                    if (buf.size() > kMergeAbove) sym_merge(buf);
                    continue;
                }
                TAMD_PROF_SCOPE(kElimFold);
                const RowId p = fold_low_levels(ctx_->rows, ctx_->pb, buf, 3, rec->bytes, row_bytes_);
                if (p != kNoRow) ctx_->temps.push_back(p);
                continue;
            }

            const uint8_t rx = row_value(m.Row);
            {
            TAMD_PROF_SCOPE(kElimSums);
            for (unsigned l = 0; l < kLanes; ++l) {
                const unsigned op = row_opcode(l, m.Row);
                if (!op) continue;
                LaneSums& c = get_lane(l, ee);
                const uint32_t n = c.bytes < rbytes ? c.bytes : rbytes;
                if (!n) continue;
                uint8_t k[3];
                opcode_coefs(op, rx, k);  // sums and RX * product sums in one read
                c.read(ctx_->rows, ctx_->ex, buf, k, n, &ctx_->pb, ctx_->short_scans);
            }
            }
            TAMD_PROF_SCOPE(kElimPairs);
            // LDPC pairs; the product half takes its RX factor right away (the reference adds
            // RX * product after the loop, SiameseDecoder.cpp:1029-1047: the same terms)
            Pcg32 prng;
            prng.seed(m.Row, m.LDPCCount);
            const uint32_t pairs = (m.LDPCCount + kPairRate - 1) / kPairRate;
            const FastMod ldpc_mod(m.LDPCCount);
            for (uint32_t i = 0; i < pairs; ++i) {
                RowId row;
                uint32_t b;
                const uint32_t e1 = es + ldpc_mod(prng.next());
                if (packet(e1, row, b)) read_original(row, b < rbytes ? b : rbytes, 1, buf);
                const uint32_t erx = es + ldpc_mod(prng.next());
                if (packet(erx, row, b)) read_original(row, b < rbytes ? b : rbytes, rx, buf);
            }
        }
        if (ctx_->oom) return false;
        // (every term is already clipped to rec->bytes: the row itself, lane reads at
        // min(sum bytes, rbytes), originals at min(bytes, rbytes))
        // Fold everything already in memory into one partial row so the triangular solve and
        // any later reader in this program touch one row instead of the whole elimination.
        // A single unknown needs no triangular solve: back substitution scales the terms
        // straight into the recovered row.  Short lists are not merged: a row named twice by
        // the pairs is just read twice (GF(2^8) sums are linear).  Long ones are -- they come
        // from inlined expansions of rows recovered in this program, which nest, and unmerged
        // duplicates would compound from one recovery to the next.
        if (cr_.lost_count == 1) {
            if (buf.size() > kMergeAbove) sym_merge(buf);
            continue;
        }
        TAMD_PROF_SCOPE(kElimFold);
        const RowId p = fold_low_levels(ctx_->rows, ctx_->pb, buf, 3, rec->bytes, row_bytes_);
        if (p != kNoRow) ctx_->temps.push_back(p);
    }
    return !disabled_ && !ctx_->oom;
}

// A Siamese row's elimination straight from the packets (the decoder's counterpart of the
// encoder's direct dense ranges, Encoder::defer_dense).  The reference subtracts the lanes' running
// sums over the row's sum range [sum_elem, ee) (SiameseDecoder.cpp:900-1028, GetSum :1680-1739)
// and then its LDPC pairs (:1029-1047).  A lane sum holds every element of its lane in that range
// that has data when it is read -- received, or recovered and plugged in (PlugSumHoles) -- each
// zero-padded to the longest and read clipped to the row's length, so the same value is
//   sum over known elements j in [sum_elem, ee) of coef(lane opcode of j, cx_j, RX) * clip(x_j),
// one DENSE run term per run of received packets (coefficients computed on the device, the pairs
// that land in the run folded in as ADJ additions) and one term per other known element.  Valid
// while sum_elem is in the window: then no element the sums would hold has been removed (a
// removal only ever cuts a prefix, and advances the lanes past it first).  The lane sums stay as
// the reference leaves them (start_sums / reset_sums ran) but are not advanced here: a later
// lane read accumulates from where they stand.  Returns false, with nothing appended, when the
// range is long or broken into short runs (C ABI adds are one record each): the lanes are used.
bool Decoder::eliminate_direct(Recovery* rec, uint32_t sum_elem, Sym& buf) {
    const RecoveryMeta m = rec->meta;
    const uint32_t es = rec->element_start, ee = rec->element_end;
    if (ee <= sum_elem || ee - sum_elem > Encoder::kDirectMax || ee > count_) return false;
    TAMD_PROF_SCOPE(kElimSums);
    const uint32_t rbytes = rec->bytes;
    // the range's records: runs of segment packets and single known elements
    drun_.clear();
    uint32_t singles = 0;
    for (uint32_t j = sum_elem; j < ee;) {
        const uint32_t id = seg_id(j);
        if (id != kSingle) {
            const Segment& sg = segs_[id - seg_base_];
            const uint32_t k = j + base_ - sg.first;
            const uint32_t stop = std::min(sg.end() - base_, ee);
            if (sg.bytes) drun_.push_back(DirectRun{j, stop - j, sg.off(k), sg.stride, std::min(sg.bytes, rbytes),
                                                    col_add(sg.column0, k), kNoRow});
            j = stop;
            continue;
        }
        const StoredOriginal& o = elem(j);
        if (o.bytes > 0) {
            drun_.push_back(DirectRun{j, 0, 0, 0, std::min(o.bytes, rbytes), to_column(j), o.row});
            ++singles;
        }
        ++j;
    }
    if (drun_.size() * Encoder::kDirectMinRun > ee - sum_elem) {
        drun_.clear();
        return false;
    }
    // LDPC pairs (element << 8 | coefficient): those on a run's packets become its ADJ additions
    // (sorted), the others are read as rows (only when the element has data).  The pairs span the
    // row's whole unacknowledged window, mostly wider than the sum range: the ones outside it are
    // read right away and only the rest are sorted.
    const uint8_t rx = row_value(m.Row);
    auto loose_pair = [&](uint64_t pr) {
        RowId row;
        uint32_t b;
        if (packet((uint32_t)(pr >> 8), row, b)) read_original(row, b < rbytes ? b : rbytes, (uint8_t)pr, buf);
    };
    Pcg32 prng;
    prng.seed(m.Row, m.LDPCCount);
    const uint32_t pairs = (m.LDPCCount + kPairRate - 1) / kPairRate;
    const FastMod ldpc_mod(m.LDPCCount);
    const uint32_t span0 = drun_.empty() ? 0u : drun_.front().e0;
    const uint32_t span1 = drun_.empty() ? 0u : drun_.back().e0 + (drun_.back().n ? drun_.back().n : 1u);
    dpairs_.clear();
    for (uint32_t i = 0; i < 2 * pairs; ++i) {
        const uint64_t pr = (uint64_t)(es + ldpc_mod(prng.next())) << 8 | (i & 1u ? rx : 1u);
        const uint32_t e = (uint32_t)(pr >> 8);
        if (e >= span0 && e < span1) dpairs_.push_back(pr);
        else loose_pair(pr);
    }
    std::sort(dpairs_.begin(), dpairs_.end());
    uint64_t ops = 0;
    uint8_t lk[kLanes][3];
    for (unsigned l = 0; l < kLanes; ++l) {
        const unsigned op = row_opcode(l, m.Row);
        ops |= (uint64_t)op << (6 * l);
        opcode_coefs(op, rx, lk[l]);
    }
    // Batched sessions (Context::dense_split) cut the range into chunks of `split` elements from
    // sum_elem, each one op that stores its partial sum (level 1, a shareable combine) and enters
    // the row as one term: one work item never walks hundreds of packets (a launch's tail), as
    // the encoder's chunked dense ranges.  Otherwise each run is one run term of the row.
    static const int split_env = getenv("TONK_AMD_DEC_SPLIT") ? atoi(getenv("TONK_AMD_DEC_SPLIT")) : -1;  // (A/B)
    const uint32_t split = split_env >= 0 && ctx_->dense_split ? (uint32_t)split_env : ctx_->dense_split;
    const bool chunked = split && ee - sum_elem > split;
    ProgramBuilder& pb = ctx_->pb;
    uint32_t chunk = ~0u;
    RowId part = kNoRow;
    auto close_chunk = [&]() {
        if (part == kNoRow) return;
        pb.finish_combine(part, rbytes, nullptr, 0);
        buf.push_back(Term{part, rbytes, 1});
        part = kNoRow;
    };
    size_t pi = 0;
    for (const DirectRun& r : drun_) {
        while (pi < dpairs_.size() && (uint32_t)(dpairs_[pi] >> 8) < r.e0) loose_pair(dpairs_[pi++]);
        if (!r.n) {  // a single known element: its dense coefficient on the host
            const uint8_t* k = lk[r.col % kLanes];
            const uint8_t cx = column_value(r.col);
            const uint8_t c = (uint8_t)(k[0] ^ gf_mul(k[1], cx) ^ gf_mul(k[2], gf_sqr(cx)));
            if (c) read_original(r.row, r.len, c, buf);
            continue;
        }
        for (uint32_t a = r.e0, end = r.e0 + r.n; a < end;) {
            const uint32_t c = chunked ? (a - sum_elem) / split : 0u;
            const uint32_t b = chunked ? std::min(end, sum_elem + (c + 1) * split) : end;
            dadj_.clear();
            for (; pi < dpairs_.size() && (uint32_t)(dpairs_[pi] >> 8) < b; ++pi)
                dadj_.push_back(((uint32_t)(dpairs_[pi] >> 8) - a) << 16 | (uint32_t)(dpairs_[pi] & 0xffu) << 8);
            const uint32_t off = r.off + (a - r.e0) * r.stride, col = col_add(r.col, a - r.e0);
            if (!chunked) {
                buf.push_back(pb.dense_run_term(off, r.stride, b - a, col, ops, rx, dadj_.data(),
                                                (uint32_t)dadj_.size(), r.len));
            } else {
                if (c != chunk) {
                    close_chunk();
                    part = ctx_->alloc_temp(rbytes);
                    if (part == kNoRow) return true;  // (ctx_->oom: the caller disables the decoder)
                    chunk = c;
                    pb.begin_op();
                }
                pb.op_accr_dense(off, r.stride, b - a, r.len, col, ops, rx, dadj_.data(), (uint32_t)dadj_.size());
            }
            a = b;
        }
    }
    close_chunk();
    while (pi < dpairs_.size()) loose_pair(dpairs_[pi++]);
    (void)singles;
    return true;
}

// Decoder::MultiplyLowerTriangle (:1065-1104), in coefficient space.  The reference adds row
// ci (times the GE multiplier) into every later row; here those row operations run on the
// L x L coefficients of the eliminated rows (tri_), which is O(L^3) byte operations instead of
// O(L^3) symbolic term operations, and the rows' byte lengths follow the reference's
// GrowZeroPadded.  Row ci's terms never reach past its length, so no clipping is lost.
bool Decoder::multiply_lower_triangle() {
    const uint32_t L = cr_.lost_count;
    tri_.assign((size_t)L * L, 0);
    tri_b_.resize(L);
    for (uint32_t i = 0; i < L; ++i) {
        tri_[(size_t)i * L + i] = 1;
        Recovery* r = mrows_[pivots_[i]].rec;
        if (L > 1) sym_merge(r->buf);  // (one unknown: merged by eliminate_original_data)
        tri_b_[i] = r->bytes;
    }
    for (uint32_t ci = 0; ci + 1 < L; ++ci) {
        const uint8_t* src = &tri_[(size_t)ci * L];
        for (uint32_t cj = ci + 1; cj < L; ++cj) {
            const uint8_t y = mat(pivots_[cj], ci);
            if (y == 0) continue;
            if (tri_b_[cj] < tri_b_[ci]) tri_b_[cj] = tri_b_[ci];  // GrowZeroPadded
            uint8_t* dst = &tri_[(size_t)cj * L];
            const uint8_t* my = g_gf.mul[y];
            for (uint32_t k = 0; k <= ci; ++k)
                if (src[k]) dst[k] ^= my[src[k]];
        }
    }
    return true;
}

// Decoder::BackSubstitution (:1106-1238).  Right to left, the recovered value of column ci is
// inv(diag) * (row ci after the triangle + sum over later columns cj of M[ci][cj] * value_cj
// clipped to row ci's length), exactly the reference's sequence of GF row operations and
// min-length adds, accumulated as groups (eliminated row k, clip length, coefficient) -- one
// group per (k, distinct length) -- and expanded into terms once per recovered row.  The
// recovered length is data dependent (the framed header inside the recovered bytes); the
// symbolic solve uses the recovery row length, which only adds zero bytes, and the exact length
// is read back with the data.
Result Decoder::back_substitution() {
    const uint32_t L = cr_.lost_count;
    recovered_.assign(L, RecoveredPacket());
    if (L == 1) return back_substitution_one();
    tri_clips_.assign(tri_b_.begin(), tri_b_.end());
    std::sort(tri_clips_.begin(), tri_clips_.end());
    tri_clips_.erase(std::unique(tri_clips_.begin(), tri_clips_.end()), tri_clips_.end());
    const uint32_t D = (uint32_t)tri_clips_.size();
    auto clip_index = [this](uint32_t len) {
        return (uint32_t)(std::lower_bound(tri_clips_.begin(), tri_clips_.end(), len) - tri_clips_.begin());
    };
    tri_groups_.clear();
    tri_gstart_.assign((size_t)L + 1, 0);  // groups of column c: [tri_gstart_[c], tri_gstart_[c + 1])
    // (columns are solved right to left; groups are appended in that order, so column c's
    // range is recorded as it is produced and located through gpos)
    std::vector<uint32_t>& gpos = tri_gstart_;
    std::vector<uint32_t> gend(L, 0);
    tri_acc_.resize((size_t)L * D);
    // Every recovered value is a combination of up to L eliminated rows.  From
    // Context::backsub_rows unknowns on, each eliminated row with more than one term is first
    // materialized (one op reading its terms once) and the values combine those rows: Sum|buf| +
    // L^2 row reads on the device and term copies on the host, instead of up to L * Sum|buf| of
    // both, for one more level.
    if (L >= ctx_->backsub_rows) {
        for (uint32_t k = 0; k < L; ++k) {
            Recovery* r = mrows_[pivots_[k]].rec;
            if (r->buf.size() <= 1) continue;
            const RowId row = ctx_->alloc_temp(r->bytes);
            if (row == kNoRow) { disabled_ = true; return kDisabled; }
            ctx_->pb.combine(row, r->buf.data(), r->buf.size(), r->bytes);
            r->buf.clear();
            r->buf.push_back(Term{row, r->bytes, 1});
        }
    }
    bool iterate = false;
    for (int ci = (int)L - 1; ci >= 0; --ci) {
        const uint32_t ri = pivots_[ci];
        const uint8_t y = mat(ri, (uint32_t)ci);
        if (y == 0) { disabled_ = true; return kDisabled; }
        const uint8_t inv_y = gf_inv(y);
        const uint32_t bytes = tri_b_[ci];
        const uint32_t bidx = clip_index(bytes);

        std::fill(tri_acc_.begin(), tri_acc_.end(), 0);
        const uint8_t* trow = &tri_[(size_t)ci * L];
        for (uint32_t k = 0; k <= (uint32_t)ci; ++k)
            if (trow[k]) tri_acc_[(size_t)k * D + bidx] ^= trow[k];
        for (uint32_t cj = ci + 1; cj < L; ++cj) {
            const uint8_t x = mat(ri, cj);
            if (x == 0) continue;
            const uint8_t* mx = g_gf.mul[x];
            for (uint32_t g = gpos[cj]; g < gend[cj]; ++g) {
                const Group& gr = tri_groups_[g];
                const uint32_t c = gr.clip < bidx ? gr.clip : bidx;  // min(length) as index
                tri_acc_[(size_t)gr.k * D + c] ^= mx[gr.coef];
            }
        }
        gpos[ci] = (uint32_t)tri_groups_.size();
        const uint8_t* my = g_gf.mul[inv_y];
        for (uint32_t k = 0; k < L; ++k)
            for (uint32_t c = 0; c < D; ++c) {
                const uint8_t a = tri_acc_[(size_t)k * D + c];
                if (a) tri_groups_.push_back(Group{k, c, my[a]});
            }
        gend[ci] = (uint32_t)tri_groups_.size();

        Sym& value = value_;
        value.clear();
        for (uint32_t g = gpos[ci]; g < gend[ci]; ++g) {
            const Group& gr = tri_groups_[g];
            sym_add(value, mrows_[pivots_[gr.k]].rec->buf, tri_clips_[gr.clip], gr.coef);
        }
        sym_merge(value);
        if (!store_recovered((uint32_t)ci, value, bytes, iterate)) return kDisabled;
    }
    return finish_solve(iterate);
}

// One unknown (the common case at low loss): the recovered value is inv(diag) times the single
// eliminated row, whose terms eliminate_original_data clipped to the row's length -- the general
// path's groups reduce to that list (merged there; duplicates are harmless reads here).
Result Decoder::back_substitution_one() {
    const uint32_t ri = pivots_[0];
    const uint8_t y = mat(ri, 0);
    if (y == 0) { disabled_ = true; return kDisabled; }
    Recovery* rec = mrows_[ri].rec;
    Sym& value = value_;
    value.swap(rec->buf);  // (rec->buf is cleared below in any case)
    sym_scale(value, gf_inv(y));
    bool iterate = false;
    if (!store_recovered(0, value, tri_b_[0], iterate)) return kDisabled;
    return finish_solve(iterate);
}

// Materialize recovered column ci (one combine op) and put it into its window slot.
bool Decoder::store_recovered(uint32_t ci, Sym& value, uint32_t bytes, bool& iterate) {
    StoredOriginal* o = mcols_[ci].orig;
    const RowId out_row = ctx_->alloc(bytes);
    if (out_row == kNoRow) { disabled_ = true; return false; }
    ctx_->pb.combine(out_row, value.data(), value.size(), bytes);
    ctx_->ex.take(out_row, value);  // (value's storage is exchanged: not read again)

    drop_original(*o);
    o->row = out_row;
    o->off = ctx_->rows.offset(out_row);
    o->bytes = bytes;
    o->column = mcols_[ci].column;
    o->header_bytes = 0;
    o->owned = 1;
    o->run = 0;
    o->stride = 0;
    {
        const uint32_t e = to_element(o->column);
        subs_[e / kSubwindow]->held |= 1ull << (e % kSubwindow);
        subs_[e / kSubwindow]->singles |= 1ull << (e % kSubwindow);
    }

    RecoveredPacket& rp = recovered_[ci];
    rp.packet_num = o->column;
    rp.row = out_row;
    rp.framed_upper = bytes;
    recovered_columns_.push_back(o->column);
    iterate |= mark_got(o->column);
    return true;
}

Result Decoder::finish_solve(bool iterate) {
    const uint32_t L = cr_.lost_count;
    for (uint32_t ci = 0; ci < L; ++ci) {
        Recovery* rec = mrows_[pivots_[ci]].rec;
        rec->buf.clear();
        rec->bytes = 0;
    }
    if (!iterate) { disabled_ = true; return kDisabled; }
    iterate_next_expected(cr_.next_check_start);
    list_delete_before(next_expected_);
    if (cr_.next_check_start >= kRemoveThreshold) remove_elements();
    stats_[7]++;
    return kSuccess;
}

void Decoder::set_recovered_length(uint32_t packet_num, uint32_t framed_bytes, uint32_t header_bytes, void* host) {
    const uint32_t e = to_element(packet_num);
    if (invalid_element(e) || seg_id(e) != kSingle) { if (host && release_) release_(host, user_); return; }
    StoredOriginal& o = elem(e);
    if (o.column != packet_num || o.bytes == 0) { if (host && release_) release_(host, user_); return; }
    o.bytes = framed_bytes;
    o.header_bytes = (uint8_t)header_bytes;
    if (o.host && release_) release_(o.host, user_);
    o.host = host;
}

// Decoder::Get (:71-123)
Result Decoder::get(uint32_t packet_num, StoredOriginal** out, bool recovered_now) {
    *out = nullptr;
    if (disabled_ && !recovered_now) return kDisabled;
    const uint32_t e = to_element(packet_num);
    if (invalid_element(e)) return kNeedMoreData;
    const uint32_t id = seg_id(e);
    if (id != kSingle) {  // (a segment's packet, as a value: no host copy)
        const Segment& sg = segs_[id - seg_base_];
        const uint32_t j = e + base_ - sg.first;
        view_ = StoredOriginal();
        view_.row = sg.row(j);
        view_.off = sg.off(j);
        view_.bytes = sg.bytes;
        view_.column = packet_num;
        view_.header_bytes = sg.header_bytes;
        *out = &view_;
        return kSuccess;
    }
    StoredOriginal& o = elem(e);
    if (o.bytes <= 0) return kNeedMoreData;
    *out = &o;
    return kSuccess;
}

// Decoder::GenerateAcknowledgement (:125-255)
Result Decoder::ack(uint8_t* buffer, uint32_t limit, uint32_t* used) {
    if (disabled_) return kDisabled;
    const uint32_t wc = count_;
    if (wc == 0) { *used = 0; return kNeedMoreData; }
    uint8_t* start = buffer;
    const uint32_t nee = next_expected_;
    const uint32_t hb = put_pnum_header(to_column(nee), buffer);
    buffer += hb;
    limit -= hb;
    if (invalid_element(nee)) {
        *used = (uint32_t)(buffer - start);
        stats_[4]++;
        stats_[5] += *used;
        return kSuccess;
    }
    uint32_t off = nee;
    while (limit >= kMaxLossRangeBytes) {
        const uint32_t rs = find_next_lost(off);
        if (rs >= wc) {
            if (wc >= off) buffer += put_nack_range(wc - off, 0, buffer);
            break;
        }
        const uint32_t re = find_next_got(rs + 1);
        const uint32_t n = put_nack_range(rs - off, re - rs - 1, buffer);
        off = re + 1;
        buffer += n;
        limit -= n;
    }
    *used = (uint32_t)(buffer - start);
    stats_[4]++;
    stats_[5] += *used;
    return kSuccess;
}

// Decoder::GetStatistics (:1240-1254)
void Decoder::stats(uint64_t* out, unsigned n) {
    if (n > 11) n = 11;
    stats_[10] = ctx_->rows.bytes_in_use();
    for (unsigned i = 0; i < n; ++i) out[i] = stats_[i];
}

} // namespace tamd
