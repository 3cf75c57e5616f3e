// encoder.cpp -- Siamese encoder control plane.  Each function names the reference routine it
// restates (SiameseEncoder.cpp line numbers); byte work becomes symbolic terms (engine.h).
#include "encoder.h"
#include "prof.h"

#include <algorithm>
#include <stdlib.h>
#include <string.h>
#include <time.h>

namespace tamd {

// Test hook (tamd_set_clock): a virtual millisecond clock replacing the monotonic one.
static uint64_t (*g_clock_fn)() = nullptr;
void set_clock_source(uint64_t (*fn)()) { g_clock_fn = fn; }

// GetTimeMsec (SiameseTools.cpp:105-117): wall-clock milliseconds, the time base the reference's
// 32-bit send timestamps and RTT arithmetic run on.  Read once per original.
uint64_t time_msec() {
    if (g_clock_fn) return g_clock_fn();
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);  // gettimeofday's clock, as the reference (vDSO, no syscall)
    return (uint64_t)ts.tv_sec * 1000u + (uint64_t)ts.tv_nsec / 1000000u;
}

Encoder::Encoder(Context* ctx, uint32_t row_bytes, HostRelease release, void* user)
    : ctx_(ctx), row_bytes_(row_bytes), release_(release), user_(user) {
    // ClearWindow (SiameseEncoder.cpp:64-83)
    for (unsigned l = 0; l < kLanes; ++l) lanes_[l].next_abs = l;
    ctx_->attach(this);
}

Encoder::~Encoder() {
    pre_flush();  // snapshots already referenced by the pending program must still be written
    drop_all();
    for (unsigned l = 0; l < kLanes; ++l) lanes_[l].sums.release(ctx_->rows);
    ctx_->detach(this);
}

void Encoder::release_segment(const Segment& s, uint32_t from, uint32_t n) {
    if (s.owned)
        for (uint32_t j = from; j < from + n; ++j) ctx_->rows.free_deferred(s.row(j));
    if (s.host && release_ && from == 0 && n == s.count) release_(s.host, user_);
}

void Encoder::drop_all() {
    if (held_)
        for (size_t i = 0; i < segs_.size(); ++i) release_segment(segs_[i], 0, segs_[i].count);
    held_ = 0;
    seg_base_ += (uint32_t)segs_.size();
    segs_.clear();
    win_.clear();
    base_ = 0;
}

StoredOriginal Encoder::view(uint32_t e) const {
    const Segment& s = seg_of(e);
    const uint32_t j = e + base_ - s.first;
    StoredOriginal o;
    o.row = s.row(j);
    o.bytes = s.bytes;
    o.column = to_column(e);
    o.send_msec = win_[e].send_msec;
    o.off = s.off(j);
    o.header_bytes = s.header_bytes;
    o.owned = s.owned;
    o.host = s.host;
    return o;
}

void Encoder::pre_flush() {
    emit_cauchy_group();
    emit_dense_group();
    for (unsigned l = 0; l < kLanes; ++l) lanes_[l].sums.flush(ctx_->rows, ctx_->pb, ctx_->ex);
}

void Encoder::append(const RowId* rows, uint32_t k, uint32_t framed_bytes, uint32_t header_bytes, uint8_t owned,
                     void* host, uint32_t now, uint64_t layout) {
    const RowTable& rt = ctx_->rows;
    uint32_t e_abs = base_ + (uint32_t)win_.size();
    uint32_t col = next_column_;
    win_.reserve_more(k);
    Slot* wb = win_.slot_base();
    const size_t mask = win_.slot_mask();
    size_t idx = win_.slot_index(win_.size());
    // Fast path: the k packets are consecutive handles at one offset stride with no column wrap
    // inside (a stretch of a session's inputs): they continue the last segment or open one, and
    // only the element slots are filled.
    if (k >= 2 && !host && col + k - 1 < kColumnPeriod && col != 0 && (layout || consecutive_handles(rows, k))) {
        const uint32_t o0 = layout ? (uint32_t)(layout >> 32) : rt.offset(rows[0]);
        const uint32_t o1 = layout ? o0 + (uint32_t)layout : rt.offset(rows[1]);
        const uint32_t stride = o1 - o0;
        if (o1 > o0 && (layout || rt.affine(rows[0], k, stride))) {
            Segment* last = segs_.empty() ? nullptr : &segs_.back();
            const bool cont = last && !last->host && last->row0 != kNoRow && last->end() == e_abs &&
                              last->bytes == framed_bytes && last->header_bytes == header_bytes &&
                              last->owned == owned && rows[0] == last->row0 + last->count && o0 > last->off0 &&
                              (last->count == 1 ? o0 - last->off0 == stride
                                                : last->stride == stride && o0 == last->off(last->count));
            if (cont) {
                last->stride = stride;
                last->count += k;
            } else {
                Segment sg;
                sg.first = e_abs;
                sg.count = k;
                sg.row0 = rows[0];
                sg.off0 = o0;
                sg.stride = stride;
                sg.bytes = framed_bytes;
                sg.column0 = col;
                sg.header_bytes = (uint8_t)header_bytes;
                sg.owned = owned;
                segs_.push_back(sg);
                if (owned) ++held_;
            }
            const Slot v{seg_base_ + (uint32_t)segs_.size() - 1, now};
            for (uint32_t x = 0; x < k; ++x) wb[(idx + x) & mask] = v;
            win_.commit(k);
            return;
        }
    }
    uint32_t j = 0;
    while (j < k) {
        // extend the last segment when this packet continues it, else open one
        Segment* last = segs_.empty() ? nullptr : &segs_.back();
        const RowId r = rows[j];
        const uint32_t off = rt.offset(r);
        const bool cont = last && !host && !last->host && last->row0 != kNoRow && last->end() == e_abs &&
                          last->bytes == framed_bytes && last->header_bytes == header_bytes && last->owned == owned &&
                          r == last->row0 + last->count && off > last->off0 && col != 0 &&
                          (last->count == 1 || off == last->off(last->count));
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
            sg.host = host;
            segs_.push_back(sg);
            if (owned || host) ++held_;
            last = &segs_.back();
        }
        const uint32_t id = seg_base_ + (uint32_t)segs_.size() - 1;
        wb[idx] = Slot{id, now};
        idx = (idx + 1) & mask;
        ++e_abs;
        col = col_inc(col);
        ++j;
        // the rest of the run while rows keep both strides (one contiguous scan of the handles'
        // offsets): only the per-element slot is written
        if (last->count >= 2) {
            uint32_t n = last->count;
            while (j < k && rows[j] == last->row0 + n && col != 0 && rt.offset(rows[j]) == last->off(n)) {
                wb[idx] = Slot{id, now};
                idx = (idx + 1) & mask;
                ++n;
                ++j;
                col = col_inc(col);
            }
            e_abs += n - last->count;
            last->count = n;
        }
    }
    win_.commit(k);
}

// EncoderPacketWindow::Add (SiameseEncoder.cpp:85-161)
Result Encoder::add(RowId row, uint32_t framed_bytes, uint32_t header_bytes, uint32_t payload_bytes,
                    void* host, uint32_t* packet_num, bool borrowed) {
    if (disabled_) return kDisabled;
    if (remaining_slots() <= 0) return kMaxPacketsReached;
    *packet_num = add_first(row, framed_bytes, header_bytes, payload_bytes, host, borrowed);
    return kSuccess;
}

// The window part of Add for one packet: a new window when the previous one is empty (elements
// below column % kLanes of a fresh window are placeholders: only the RTT scan reads them, and only
// their send timestamps), then the packet at the window end.
uint32_t Encoder::add_first(RowId row, uint32_t framed_bytes, uint32_t header_bytes, uint32_t payload_bytes,
                            void* host, bool borrowed) {
    const uint32_t column = next_column_;
    const uint32_t now = (uint32_t)now_msec();
    if (count_ > 0) {
        ++count_;
    } else {
        start_new_window(column);
        const uint32_t element = column % kLanes;
        if (element) {
            Segment ph;
            ph.first = base_;
            ph.count = element;
            ph.column0 = column - element;
            segs_.push_back(ph);
            for (uint32_t e = 0; e < element; ++e)
                win_.push_back(Slot{seg_base_ + (uint32_t)segs_.size() - 1, placeholder_msec_[e]});
        }
    }
    append(&row, 1, framed_bytes, header_bytes, borrowed ? 0 : 1, host, now);
    next_column_ = col_inc(next_column_);
    Lane& lane = lanes_[column % kLanes];
    if (lane.longest < framed_bytes) lane.longest = framed_bytes;
    if (longest_ < framed_bytes) longest_ = framed_bytes;
    stats_[0]++;
    stats_[1] += payload_bytes;
    return column;
}

// k consecutive add() calls that all succeed.
bool Encoder::add_run(const RowId* rows, uint32_t k, uint32_t framed_bytes, uint32_t header_bytes,
                      uint32_t payload_bytes, bool borrowed, uint32_t* first_col, uint64_t layout) {
    if (disabled_ || remaining_slots() < k || !k) return false;
    // A first add that starts a window goes alone; the rest (all k when the window is open)
    // append at once (count_ > 0, element == count_).
    uint32_t skip = 0;
    if (count_ == 0) {
        *first_col = add_first(rows[0], framed_bytes, header_bytes, payload_bytes, nullptr, borrowed);
        if (k == 1) return true;
        skip = 1;
    } else {
        *first_col = next_column_;
    }
    const uint32_t m = k - skip;
    append(rows + skip, m, framed_bytes, header_bytes, borrowed ? 0 : 1, nullptr, (uint32_t)now_msec(),
           layout && skip ? layout + ((layout & 0xffffffffull) << 32) : layout);  // (rows + 1: one stride on)
    count_ += m;
    const uint32_t first = next_column_;
    next_column_ = col_add(next_column_, m);
    // every lane one of these columns fell on (all m have the same length)
    for (uint32_t j = 0; j < m && j < kLanes; ++j) {
        Lane& lane = lanes_[(first + j) % kLanes];
        if (lane.longest < framed_bytes) lane.longest = framed_bytes;
    }
    if (longest_ < framed_bytes) longest_ = framed_bytes;
    stats_[0] += m;
    stats_[1] += (uint64_t)payload_bytes * m;
    return true;
}

// EncoderPacketWindow::StartNewWindow (SiameseEncoder.cpp:163-181)
void Encoder::start_new_window(uint32_t column) {
    // Everything from the previous window is unreachable once Count reached zero (only the send
    // timestamps of its first elements stay visible to the RTT scan, see placeholder_msec_).
    for (uint32_t e = 0; e < kLanes; ++e) placeholder_msec_[e] = e < win_.size() ? win_[e].send_msec : placeholder_msec_[e];
    ++window_gen_;  // (a pending Cauchy group does not extend into the new window)
    drop_all();
    const uint32_t element = column % kLanes;
    column_start_ = column - element;
    sum_start_ = element;
    sum_end_ = element;
    first_unremoved_ = element;
    count_ = element + 1;
    longest_ = 0;
    for (unsigned l = 0; l < kLanes; ++l) lanes_[l].longest = 0;
}

// EncoderPacketWindow::RemoveBefore (SiameseEncoder.cpp:183-216)
void Encoder::remove_before(uint32_t first_kept_column) {
    if (disabled_) return;
    const uint32_t e = to_element(first_kept_column);
    if (e >= count_) {
        if (!col_delta_negative(e)) count_ = 0;  // removed everything
    } else if (first_unremoved_ < e) {
        first_unremoved_ = e;
    }
}

// EncoderPacketWindow::ResetSums (SiameseEncoder.cpp:218-237)
void Encoder::reset_sums(uint32_t element_start) {
    for (unsigned l = 0; l < kLanes; ++l) {
        lanes_[l].next_abs = base_ + next_lane_element(element_start, l);
        lanes_[l].sums.reset(ctx_->rows);
    }
    sum_start_ = element_start;
    sum_end_ = element_start;
    sum_column_start_ = to_column(element_start);
    sum_erased_ = 0;
    drop_segments_below(base_);  // (segments kept for the previous sums)
}

void Encoder::drop_segments_below(uint32_t drop) {
    while (!segs_.empty() && (int32_t)(segs_.front().end() - drop) <= 0) {
        const Segment& f = segs_.front();
        if (f.owned || f.host) {
            release_segment(f, 0, f.count);
            --held_;
        }
        segs_.pop_front(1);
        ++seg_base_;
    }
    if (!segs_.empty() && (int32_t)(segs_.front().first - drop) < 0) {
        Segment& f = segs_.front();
        const uint32_t d = drop - f.first;
        release_segment(f, 0, d);  // (a straddling segment holds no host copy: count > 1)
        f.first = drop;
        f.count -= d;
        if (f.row0 != kNoRow) f.row0 += d;
        f.off0 += d * f.stride;
        f.column0 = col_add(f.column0, d);
    }
}

// EncoderPacketWindow::RemoveElements (SiameseEncoder.cpp:239-357)
void Encoder::remove_elements() {
    TAMD_PROF_SCOPE(kEncRemove);
    const uint32_t first_kept_sub = first_unremoved_ / kSubwindow;
    const uint32_t removed = first_kept_sub * kSubwindow;

    // While the running sums are active, the lanes accumulate lazily (the reference advances them
    // here, GetSum up to the removed elements): the segments of the sum range are kept -- with the
    // rows they own -- until the sums reset, so a later lane read (or a direct dense read) still
    // finds every packet of the range.
    const uint32_t cut = base_ + removed;
    uint32_t drop = cut;
    if (sum_end_ > sum_start_) {
        const uint32_t keep = sum_abs_start();
        if ((int32_t)(keep - drop) < 0) drop = keep;
        if (removed > sum_start_) sum_erased_ += removed - sum_start_;
        sum_end_ = sum_end_ > removed ? sum_end_ - removed : 0;
        sum_start_ = sum_start_ > removed ? sum_start_ - removed : 0;
    }

    // segments below `drop` leave (what they own is released); one that straddles it keeps its
    // later packets
    drop_segments_below(drop);
    win_.pop_front(removed);
    base_ = cut;
    count_ -= removed;
    column_start_ = to_column(removed);
    first_unremoved_ -= removed;

    // longest packet of the unacknowledged elements, overall and per lane (segment by segment)
    uint32_t longest = 0, lane_longest[kLanes] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (first_unremoved_ < count_) {
        const uint32_t lo = base_ + first_unremoved_, hi = base_ + count_;
        for (uint32_t i = win_[first_unremoved_].seg - seg_base_; i < segs_.size(); ++i) {
            const Segment& sg = segs_[i];
            if (sg.first >= hi) break;
            const uint32_t a = sg.first > lo ? sg.first : lo, b = sg.end() < hi ? sg.end() : hi;
            if (a >= b || !sg.bytes) continue;
            if (longest < sg.bytes) longest = sg.bytes;
            for (uint32_t x = a; x < b && x < a + kLanes; ++x) {
                const uint32_t l = (x - base_) % kLanes;
                if (lane_longest[l] < sg.bytes) lane_longest[l] = sg.bytes;
            }
        }
    }
    longest_ = longest;
    for (unsigned l = 0; l < kLanes; ++l) lanes_[l].longest = lane_longest[l];

    if (sum_end_ <= sum_start_) reset_sums(first_unremoved_);
}

// EncoderPacketWindow::GetSum (SiameseEncoder.cpp:359-418), for the lane's three sums at once.
// The lane's packets in a segment are every kLanes-th of it: one strided run per segment.  The
// lane may start before the window (segments kept for the sums, remove_elements).
LaneSums& Encoder::get_lane(uint32_t lane_index, uint32_t element_end) {
    Lane& lane = lanes_[lane_index];
    LaneSums& sums = lane.sums;
    uint32_t a = lane.next_abs;
    const uint32_t end = base_ + element_end;
    if ((int32_t)(end - a) > 0) {
        if (lane.longest > 0) sums.grow(lane.longest);
        size_t si = seg_index_at(a);
        do {
            const Segment& sg = segs_[si];
            const uint32_t j = a - sg.first;
            const uint32_t stop = (int32_t)(sg.end() - end) < 0 ? sg.end() : end;
            const uint32_t n = (stop - 1 - a) / kLanes + 1;  // lane packets in [a, stop)
            if (sg.bytes) {
                sums.grow(sg.bytes);
                sums.accumulate_run_level0(sg.row(j), sg.off(j), sg.bytes, col_add(sg.column0, j), n,
                                           sg.stride * kLanes);
            }
            a += n * kLanes;
            while (si + 1 < segs_.size() && (int32_t)(segs_[si].end() - a) <= 0) ++si;
        } while ((int32_t)(end - a) > 0);
        lane.next_abs = a;
    }
    return sums;
}

// ---- acknowledgements (SiameseEncoder.cpp:514-800) ----

bool Encoder::on_ack_data(const uint8_t* data, uint32_t bytes) {
    unsigned next = 0;
    const int hb = get_pnum_header(data, (int)bytes, next);
    if (hb < 1) return false;
    data += hb;
    bytes -= (uint32_t)hb;

    if (col_delta_negative(col_sub(next, ack_.next_expected))) return true;  // out of order

    if (ack_.next_expected == next && ack_.have_data && bytes == ack_.data_bytes &&
        (bytes == 0 || memcmp(data, ack_.data.data(), bytes) == 0))
        return true;  // duplicate

    ack_.next_expected = next;
    ack_.offset = 0;
    ack_.loss_column = next;
    ack_.loss_count = 0;
    ack_.data_bytes = bytes;
    if (bytes > 0) {
        ack_.data.assign(data, data + bytes);
        ack_.data.resize((size_t)bytes + 8, 0);
        ack_.have_data = true;
        if (!decode_next_range()) return false;
    }
    update_rto();
    remove_before(ack_.next_expected);
    return true;
}

// WindowedMinMax<.., WindowedMaxCompare>::Update (SiameseTools.h:184-235)
void Encoder::rtt_update(uint32_t value, uint64_t now, uint64_t window) {
    auto* s = ack_.max_rtt;
    auto expired = [&](int i, uint64_t w) { return (uint64_t)(now - s[i].ts) > w; };
    if (s[0].value == 0 || value >= s[0].value || expired(2, window)) {
        s[0].value = s[1].value = s[2].value = value;
        s[0].ts = s[1].ts = s[2].ts = now;
        return;
    }
    if (value >= s[1].value) { s[1].value = s[2].value = value; s[1].ts = s[2].ts = now; }
    else if (value >= s[2].value) { s[2].value = value; s[2].ts = now; }
    if (expired(0, window)) {
        if (expired(1, window)) { s[0] = s[2]; s[1].value = value; s[1].ts = now; }
        else { s[0] = s[1]; s[1] = s[2]; }
        s[2].value = value;
        s[2].ts = now;
        return;
    }
    if (s[1].value == s[0].value && expired(1, window / 4)) {
        s[1].value = s[2].value = value;
        s[1].ts = s[2].ts = now;
        return;
    }
    if (s[2].value == s[1].value && expired(2, window / 2)) { s[2].value = value; s[2].ts = now; }
}

// EncoderAcknowledgementState::UpdateRTO (SiameseEncoder.cpp:584-723)
void Encoder::update_rto() {
    const uint32_t window_count = count_;
    uint32_t first_loss = to_element(ack_.next_expected);
    if (first_loss >= window_count) return;

    const uint64_t now64 = now_msec();
    const uint32_t now = (uint32_t)now64;
    uint32_t longest = 0;

    uint32_t element = to_element(ack_.next_rto_column);
    if (element >= window_count) element = first_unremoved_;

    for (; element < first_loss; ++element) {
        const int32_t d = (int32_t)(now - win_[element].send_msec);
        if ((uint32_t)d > longest && d > 0) longest = (uint32_t)d;
    }

    uint32_t remaining = ack_.data_bytes;
    const uint8_t* data = ack_.data.data();
    while (remaining > 0) {
        unsigned rel = 0, lossM1 = 0;
        const int n = get_nack_range(data, remaining + 8, rel, lossM1);
        if (n < 0 || n > (int)remaining) return;
        data += n;
        remaining -= (uint32_t)n;
        if (element + 1 < first_loss) element = first_loss - 1;
        first_loss += rel;
        for (; element < first_loss; ++element) {
            if (element >= window_count) return;
            const int32_t d = (int32_t)(now - win_[element].send_msec);
            if ((uint32_t)d > longest && d > 0) longest = (uint32_t)d;
        }
        first_loss += lossM1 + 2;
    }
    ack_.next_rto_column = to_column(element);
    if (longest <= 0) return;

    uint64_t window = (uint64_t)ack_.rto_msec * 2;
    if (window < 100) window = 100;
    else if (window > 4000) window = 4000;
    rtt_update(longest, now64, window);
    ack_.rto_msec = (ack_.max_rtt[0].value * 3) / 2;
    if (ack_.rto_msec < 20) ack_.rto_msec = 20;
}

// EncoderAcknowledgementState::DecodeNextRange (SiameseEncoder.cpp:725-755)
bool Encoder::decode_next_range() {
    if (ack_.offset >= ack_.data_bytes) return false;
    unsigned rel = 0, lossM1 = 0;
    const int n = get_nack_range(ack_.data.data() + ack_.offset, ack_.data_bytes + 8 - ack_.offset, rel, lossM1);
    if (n < 0) return false;
    ack_.offset += (uint32_t)n;
    if (ack_.offset > ack_.data_bytes) return false;
    ack_.loss_column = col_add(ack_.loss_column, rel);
    ack_.loss_count = lossM1 + 1;
    return true;
}

// GetNextLossColumn (SiameseEncoder.cpp:757-777)
bool Encoder::next_loss_column(uint32_t& column) {
    if (ack_.loss_count <= 0) {
        ack_.loss_column = col_inc(ack_.loss_column);
        if (!decode_next_range()) return false;
    }
    column = ack_.loss_column;
    ack_.loss_column = col_inc(ack_.loss_column);
    --ack_.loss_count;
    return true;
}

// RestartLossIterator (SiameseEncoder.cpp:779-788)
void Encoder::restart_loss_iterator() {
    ack_.offset = 0;
    ack_.loss_column = ack_.next_expected;
    ack_.loss_count = 0;
    decode_next_range();
}

// Encoder::Acknowledge (SiameseEncoder.cpp:814-833)
Result Encoder::acknowledge(const uint8_t* data, uint32_t bytes, uint32_t* next_expected) {
    if (disabled_) return kDisabled;
    if (!on_ack_data(data, bytes)) return kInvalidInput;
    *next_expected = ack_.next_expected;
    stats_[6]++;
    stats_[7] += bytes;
    return kSuccess;
}

Result Encoder::attempt_retransmit(uint32_t e, StoredOriginal* out) {
    const StoredOriginal o = view(e);
    if (o.header_bytes == 0 || o.bytes <= o.header_bytes) { disabled_ = true; return kDisabled; }
    *out = o;
    stats_[4]++;
    stats_[5] += o.bytes - o.header_bytes;
    return kSuccess;
}

// Encoder::Retransmit (SiameseEncoder.cpp:877-1044)
Result Encoder::retransmit(StoredOriginal* out) {
    if (disabled_) return kDisabled;
    if (unacked() == 0) {
        ack_.found_oldest = false;
        return kNeedMoreData;
    }
    const uint32_t first = col_sub(ack_.next_expected, column_start_);
    const uint32_t count = count_;
    if (col_delta_negative(first) || first < first_unremoved_ || first >= count) return kNeedMoreData;

    const uint32_t now = (uint32_t)now_msec();
    const uint32_t rto = ack_.rto_msec;

    if (ack_.found_oldest) {
        const uint32_t e = col_sub(ack_.oldest_column, column_start_);
        if (!col_delta_negative(e) && e >= first && e < count) {
            Slot& o = win_[e];
            if ((uint32_t)(now - o.send_msec) < rto) return kNeedMoreData;
            o.send_msec = now;
            ack_.found_oldest = false;
            return attempt_retransmit(e, out);
        }
        ack_.found_oldest = false;
    }

    uint32_t nack_element = first;
    uint32_t oldest = nack_element;
    uint32_t oldest_msec = win_[oldest].send_msec;
    if ((uint32_t)(now - oldest_msec) >= rto) {
        win_[oldest].send_msec = now;
        return attempt_retransmit(oldest, out);
    }

    if (ack_.data_bytes > 0) {
        restart_loss_iterator();
        uint32_t column = 0;
        while (next_loss_column(column)) {
            nack_element = to_element(column);
            if (nack_element >= count) break;
            Slot& o = win_[nack_element];
            const uint32_t last = o.send_msec;
            if ((uint32_t)(now - last) >= rto) {
                o.send_msec = now;
                return attempt_retransmit(nack_element, out);
            }
            if ((int32_t)(oldest_msec - last) > 0) { oldest = nack_element; oldest_msec = last; }
        }
    }

    for (uint32_t e = nack_element + 1; e < count; ++e) {
        Slot& o = win_[e];
        const uint32_t last = o.send_msec;
        if ((uint32_t)(now - last) >= rto) {
            o.send_msec = now;
            return attempt_retransmit(e, out);
        }
        if ((int32_t)(oldest_msec - last) > 0) { oldest = e; oldest_msec = last; }
    }
    ack_.found_oldest = true;
    ack_.oldest_column = to_column(oldest);
    return kNeedMoreData;
}

// Encoder::Get (SiameseEncoder.cpp:1256-1294)
Result Encoder::get(uint32_t packet_num, StoredOriginal* out) {
    if (disabled_) return kDisabled;
    const uint32_t e = to_element(packet_num);
    if (e >= count_) return kNeedMoreData;
    const StoredOriginal o = view(e);
    if (o.bytes == 0) return kNeedMoreData;
    if (o.header_bytes == 0 || o.bytes <= o.header_bytes) { disabled_ = true; return kDisabled; }
    *out = o;
    return kSuccess;
}

// ---- recovery generation ----

// `terms` is consumed.  Parity and Cauchy rows name each original once (`distinct`); Siamese
// rows can repeat a row (LDPC pairs) and are merged first.
Result Encoder::emit(Sym& terms, uint32_t len, const RecoveryMeta& meta, RecoveryOut& out, bool distinct) {
    TAMD_PROF_SCOPE(kEncEmit);
    if (!distinct) sym_merge(terms);
    out.meta = meta;
    out.footer_len = put_recovery_footer(meta, out.footer);
    out.data_len = len;
    out.row = ctx_->alloc(len + out.footer_len);
    if (out.row == kNoRow) { disabled_ = true; return kDisabled; }
    ctx_->pb.combine(out.row, terms.data(), terms.size(), len, out.footer, out.footer_len);
    stats_[2]++;
    stats_[3] += out.total();
    return kSuccess;
}

// Encoder::GenerateSinglePacket (SiameseEncoder.cpp:1296-1329)
Result Encoder::generate_single(RecoveryOut& out) {
    const StoredOriginal o = view(first_unremoved_);
    RecoveryMeta m;
    m.SumCount = 1;
    m.LDPCCount = 1;
    m.ColumnStart = o.column;
    m.Row = 0;
    Sym& t = scratch_;
    t.clear();
    t.push_back(Term{o.row, o.bytes, 1});
    return emit(t, o.bytes, m, out, true);
}

// Encoder::GenerateCauchyPacket (SiameseEncoder.cpp:1334-1441)
Result Encoder::generate_cauchy(RecoveryOut& out) {
    TAMD_PROF_SCOPE(kEncCauchy);
    const uint32_t first = first_unremoved_;
    RecoveryMeta m;
    m.SumCount = unacked();
    m.LDPCCount = m.SumCount;
    m.ColumnStart = to_column(first);
    uint32_t mode, crow = 0;
    const uint32_t next_parity = to_element(next_parity_column_);
    if (next_parity <= first || col_delta_negative(next_parity)) {
        next_parity_column_ = col_add(m.ColumnStart, m.SumCount);
        m.Row = 0;
        mode = TAMD_R_CONST;  // parity row: every coefficient 1
    } else {
        crow = next_cauchy_row_;
        m.Row = crow + 1;
        if (++next_cauchy_row_ >= kCauchyMaxRows) next_cauchy_row_ = 0;
        mode = TAMD_R_CAUCHY;  // CauchyElement(crow, column mod 64)
    }

    // The window's originals (level-0 rows): one ACCR per segment (a run of equally long packets
    // at a fixed row stride), clipped to the unacknowledged range.
    std::vector<Run>& runs = runs_;
    runs.clear();
    uint32_t used = 0;
    {
        const uint32_t lo = base_ + first, hi = base_ + count_;
        for (uint32_t i = win_[first].seg - seg_base_; i < segs_.size(); ++i) {
            const Segment& sg = segs_[i];
            if (sg.first >= hi) break;
            const uint32_t a = sg.first > lo ? sg.first : lo, b = sg.end() < hi ? sg.end() : hi;
            if (a >= b || !sg.bytes) continue;
            const uint32_t j = a - sg.first;
            if (used < sg.bytes) used = sg.bytes;
            runs.push_back(Run{sg.row(j), sg.off(j), sg.stride, b - a, sg.bytes, col_add(sg.column0, j)});
        }
    }

    out.meta = m;
    out.footer_len = put_recovery_footer(m, out.footer);
    out.data_len = used;
    out.row = ctx_->alloc(used + out.footer_len);
    if (out.row == kNoRow) { disabled_ = true; return kDisabled; }
    // The row's op is emitted with the group (at the latest by pre_flush, so within this
    // program); its readers must already see the level it will be written at.
    ctx_->rows.set_level(out.row, 1);
    static const uint32_t max_group = getenv("TONK_AMD_NO_MULTI") ? 1u : 3u;
    // (A/B knob; at most 2047: the run indices of a TARGETS word are 11-bit)
    static const uint32_t span = getenv("TONK_AMD_MULTI_SPAN")
                                     ? std::min<uint32_t>(2047u, std::max(1, atoi(getenv("TONK_AMD_MULTI_SPAN"))))
                                     : kGroupSpan;
    const uint32_t end_col = to_column(count_);
    // A row over a long window stays a pure combine of its own (the executor shares those across
    // a workgroup); a group is one wave's chain, and a long one would set the launch's tail.
    // (and rows over windows of short runs -- the C ABI's one-packet segments -- stay alone too:
    // a MULTI run per packet is an unbatched load each, a lone row's single packets are batched)
    const bool alone = count_ - first >= span || runs.size() * 4 > count_ - first;
    if (grp_n_ && (alone || grp_n_ >= max_group || grp_gen_ != window_gen_ ||
                   col_sub(end_col, grp_[0].first_col) >= span))
        emit_cauchy_group();
    grp_gen_ = window_gen_;
    CauchyTarget& t = grp_[grp_n_++];
    t.row = out.row;
    t.used = used;
    t.first_col = m.ColumnStart;
    t.end_col = end_col;
    t.kind = mode;
    t.param = mode == TAMD_R_CONST ? 1 : crow;
    t.flen = out.footer_len;
    memcpy(t.footer, out.footer, sizeof(t.footer));
    t.runs.swap(runs);
    if (alone) emit_cauchy_group();
    stats_[2]++;
    stats_[3] += out.total();
    return kSuccess;
}

void Encoder::emit_cauchy_group() {
    const uint32_t n = grp_n_;
    if (!n) return;
    grp_n_ = 0;
    ProgramBuilder& pb = ctx_->pb;
    pb.begin_op();
    if (n == 1) {  // a lone row: a pure combine (the executor may share it across a workgroup)
        const CauchyTarget& t = grp_[0];
        for (const Run& r : t.runs) {
            if (r.count == 1) {
                const uint8_t c = t.kind == TAMD_R_CONST ? 1 : cauchy_element(t.param, r.col % kCauchyMaxColumns);
                pb.op_acc(r.row, c, r.len);
            } else {
                pb.op_accr(t.kind, t.param, r.off, r.stride, r.count, r.len, r.col, 1);
            }
        }
        pb.finish_combine(t.row, t.used, t.footer, t.flen);
        return;
    }
    // The union of the windows in runs: row a's runs below the next row's first column.
    const uint32_t base = grp_[0].first_col;
    std::vector<Run>& u = grp_union_;
    u.clear();
    for (uint32_t a = 0; a < n; ++a) {
        const uint32_t stop = a + 1 < n ? col_sub(grp_[a + 1].first_col, base) : ~0u;
        for (const Run& r : grp_[a].runs) {
            const uint32_t at = col_sub(r.col, base);
            if (at >= stop) continue;
            Run c = r;
            if (at + c.count > stop) c.count = stop - at;
            u.push_back(c);
        }
    }
    for (const Run& r : u) {
        const uint32_t at = col_sub(r.col, base);
        uint32_t tw[3] = {0, 0, 0};
        for (uint32_t a = 0; a < n; ++a) {
            const uint32_t f = col_sub(grp_[a].first_col, base), e = col_sub(grp_[a].end_col, base);
            const uint32_t lo = f > at ? f - at : 0u;
            const uint32_t hi = e - at < r.count ? e - at : r.count;  // (e > at: within the union)
            if (e > at && lo < hi) tw[a] = grp_[a].kind | grp_[a].param << 2 | lo << 10 | hi << 21;
        }
        if (tw[0] | tw[1] | tw[2]) pb.op_accr_multi(r.off, r.stride, r.count, r.len, r.col, 1, tw);
    }
    for (uint32_t a = 0; a < n; ++a) pb.op_store(grp_[a].row, grp_[a].used, a, grp_[a].footer, grp_[a].flen);
    pb.end_op(1);
}

// Encoder::AddDenseColumns (SiameseEncoder.cpp:1046-1098)
// The product half (opcode bits 3..5) is folded in with its RX factor right here: both halves
// are clipped to the same length, so rec + RX * prod reads each lane once.
void Encoder::add_dense(uint32_t row, uint32_t recovery_bytes, Sym& rec) {
    const uint8_t rx = row_value(row);
    for (unsigned l = 0; l < kLanes; ++l) {
        const unsigned op = row_opcode(l, row);
        if (!op) continue;
        LaneSums& c = get_lane(l, count_);
        const uint32_t n = c.bytes < recovery_bytes ? c.bytes : recovery_bytes;
        if (!n) continue;
        uint8_t k[3];
        opcode_coefs(op, rx, k);
        c.read(ctx_->rows, ctx_->ex, rec, k, n, nullptr, ctx_->short_scans);
    }
    sum_end_ = count_;
}

// AddDenseColumns straight from the packets: the lane sums a Siamese row reads are sums over the
// packets of its sum range, so the row's dense part is one DENSE run per segment of that range
// (program.h), each packet weighted by its lane's opcode combination -- no lane walk, snapshot
// or carried sum.  Bytes are the same: a lane sum is its packets zero-padded to the longest, and
// each packet is clipped to the recovery length as the sum would be.  The row's LDPC pair
// columns (light_pairs) are folded into the runs' coefficients (ADJ words); a pair column no run
// covers is read as a row of its own.
//
// Rows are queued (dgrp_) and emitted by emit_dense_group: rows of one sum range share its
// packets, so up to three of them are one op per chunk, each packet loaded once for all.
bool Encoder::defer_dense(uint32_t row, uint32_t recovery_bytes, const RecoveryOut& out) {
    static const uint32_t max_group = getenv("TONK_AMD_NO_DENSE_GROUP") ? 1u : 3u;  // (A/B knob)
    // A group's op is one work item per slice (one wave, or one workgroup in small launches), so
    // its products per item are bounded as a lone row's are: packets per chunk x targets
    static const uint32_t max_work = getenv("TONK_AMD_DENSE_WORK") ? (uint32_t)atoi(getenv("TONK_AMD_DENSE_WORK"))
                                                                  : kDenseGroupWork;
    const uint32_t lo = sum_abs_start(), hi = base_ + count_;
    const uint32_t split = ctx_->dense_split;
    const uint32_t rows = split && hi - lo > split ? split : hi - lo;
    if (dgrp_n_ && (lo != dgrp_lo_ || recovery_bytes != dgrp_len_ || window_gen_ != dgrp_gen_ ||
                    rows * (dgrp_n_ + 1) > max_work))
        emit_dense_group();
    // The range's runs (a superset of the queued rows' ranges: they share `lo` and end earlier)
    std::vector<DenseRun>& runs = dgrp_runs_;
    runs.clear();
    for (size_t i = seg_index_at(lo); i < segs_.size(); ++i) {
        const Segment& sg = segs_[i];
        if ((int32_t)(sg.first - hi) >= 0) break;
        const uint32_t a = (int32_t)(sg.first - lo) > 0 ? sg.first : lo;
        const uint32_t b = (int32_t)(sg.end() - hi) < 0 ? sg.end() : hi;
        if ((int32_t)(b - a) <= 0 || !sg.bytes) continue;
        const uint32_t j = a - sg.first;
        runs.push_back(DenseRun{sg.off(j), sg.stride, b - a, sg.bytes < recovery_bytes ? sg.bytes : recovery_bytes,
                                col_add(sg.column0, j), a - lo});
    }
    if (!dgrp_n_) {
        dgrp_lo_ = lo;
        dgrp_len_ = recovery_bytes;
        dgrp_gen_ = window_gen_;
    }
    DenseTarget& t = dgrp_[dgrp_n_];
    t.row = out.row;
    t.ops = 0;
    for (unsigned l = 0; l < kLanes; ++l) t.ops |= (uint64_t)row_opcode(l, row) << (6 * l);
    t.rx = row_value(row);
    t.hi = hi - lo;
    t.flen = out.footer_len;
    memcpy(t.footer, out.footer, sizeof(t.footer));
    // pair columns as (element - lo) << 8 | coefficient: those inside a run stay (ADJ words),
    // the others are resolved to their rows now (the window may have moved on by emission)
    t.pairs.clear();
    t.loose.clear();
    size_t ri = 0;
    for (uint64_t pr : pairs_) {
        const uint32_t e = (uint32_t)(pr >> 8), rel = e - lo;
        while (ri < runs.size() && runs[ri].e0 + runs[ri].count <= rel) ++ri;
        if (rel < t.hi && ri < runs.size() && runs[ri].e0 <= rel) {
            t.pairs.push_back((uint64_t)rel << 8 | (pr & 0xffu));
        } else {
            const Segment& sg = seg_of(e - base_);
            t.loose.push_back(Term{sg.row(e - sg.first), sg.bytes, (uint8_t)(pr & 0xffu)});
        }
    }
    // partial sums: one per chunk of the range (none when it fits one)
    const uint32_t chunks = split && t.hi > split ? (t.hi + split - 1) / split : 1u;
    t.parts.clear();
    for (uint32_t c = 1; chunks > 1 && c <= chunks; ++c) {
        const RowId pr = ctx_->alloc_temp(recovery_bytes);
        if (pr == kNoRow) return false;
        t.parts.push_back(pr);
    }
    // the readers of the row see the level it will be written at (emission is within this program)
    ctx_->rows.set_level(out.row, chunks > 1 ? 2 : 1);
    if (++dgrp_n_ >= max_group) emit_dense_group();
    return true;
}

void Encoder::emit_dense_group() {
    const uint32_t n = dgrp_n_;
    if (!n) return;
    dgrp_n_ = 0;
    ProgramBuilder& pb = ctx_->pb;
    const uint32_t len = dgrp_len_, split = ctx_->dense_split;
    const uint32_t total = dgrp_[n - 1].hi;  // the last (longest) range, relative to lo
    const uint32_t step = split ? split : ~0u;
    const uint32_t chunks = split && total > split ? (total + split - 1) / split : 1u;
    const std::vector<DenseRun>& runs = dgrp_runs_;
    size_t pc[3] = {0, 0, 0};  // per target: its next pair column
    thread_local std::vector<uint32_t> adj[3];
    size_t ri = 0;
    for (uint32_t c = 0; c < chunks; ++c) {
        const uint32_t c0 = c * step, c1 = total - c0 > step ? c0 + step : total;
        uint32_t a0 = 0;  // targets a0 .. n-1 reach into this chunk (ranges are nested)
        while (a0 < n && dgrp_[a0].hi <= c0) ++a0;
        if (a0 == n) a0 = n - 1;  // (empty ranges: the stores still run)
        const uint32_t nt = n - a0;
        pb.begin_op();
        for (; ri < runs.size() && runs[ri].e0 < c1; ++ri) {
            const DenseRun& r = runs[ri];
            const uint32_t pa = r.e0 > c0 ? r.e0 : c0, pe = r.e0 + r.count < c1 ? r.e0 + r.count : c1;
            const uint32_t k = pe - pa;
            ProgramBuilder::DenseCoefs tc[3];
            for (uint32_t t = 0; t < nt; ++t) {
                const DenseTarget& d = dgrp_[a0 + t];
                const uint32_t h = d.hi > pa ? (d.hi - pa < k ? d.hi - pa : k) : 0u;
                adj[t].clear();
                while (pc[a0 + t] < d.pairs.size() && (uint32_t)(d.pairs[pc[a0 + t]] >> 8) < pa + h) {
                    const uint64_t pr = d.pairs[pc[a0 + t]++];
                    adj[t].push_back(((uint32_t)(pr >> 8) - pa) << 16 | (uint32_t)(pr & 0xffu) << 8);
                }
                tc[t] = ProgramBuilder::DenseCoefs{d.ops, d.rx, h, adj[t].data(), (uint32_t)adj[t].size()};
            }
            if (nt == 1) pb.op_accr_dense(r.off + (pa - r.e0) * r.stride, r.stride, k, r.len, col_add(r.col, pa - r.e0),
                                          tc[0].ops, tc[0].rx, tc[0].adj, tc[0].nadj);
            else pb.op_accr_dense_multi(r.off + (pa - r.e0) * r.stride, r.stride, k, r.len,
                                        col_add(r.col, pa - r.e0), tc, nt);
            if (pe < r.e0 + r.count) break;  // the run continues in the next chunk
        }
        // rows over one chunk are finished here (their loose pair columns included), the others
        // store this chunk's partial sum
        for (uint32_t t = 0; t < nt; ++t) {
            const DenseTarget& d = dgrp_[a0 + t];
            if (d.parts.empty())
                for (const Term& x : d.loose) pb.op_acc(x.row, x.coef, x.len, t);
        }
        if (nt == 1) {
            const DenseTarget& d = dgrp_[a0];
            if (d.parts.empty()) pb.finish_combine(d.row, len, d.footer, d.flen);
            else pb.finish_combine(d.parts[c], len, nullptr, 0);
        } else {
            for (uint32_t t = 0; t < nt; ++t) {
                const DenseTarget& d = dgrp_[a0 + t];
                if (d.parts.empty()) pb.op_store_shared(d.row, len, t, d.footer, d.flen);
                else pb.op_store_shared(d.parts[c], len, t, nullptr, 0);
            }
            pb.end_op(1);
        }
    }
    // rows over several chunks: their partial sums and loose pair columns (level 2)
    for (uint32_t a = 0; a < n; ++a) {
        const DenseTarget& d = dgrp_[a];
        if (d.parts.empty()) continue;
        pb.begin_op();
        for (RowId p : d.parts) pb.op_acc(p, 1, len);
        for (const Term& x : d.loose) pb.op_acc(x.row, x.coef, x.len);
        pb.finish_combine(d.row, len, d.footer, d.flen);
    }
}

// Encoder::AddLightColumns (SiameseEncoder.cpp:1100-1144).  The product half goes straight into
// the row with its RX factor (the reference multiplies the product buffer by RX and adds it,
// :1236-1240; both are clipped to the same length, and every window packet is at most
// longest_ bytes, so no clipping is needed).
void Encoder::add_light(uint32_t row, Sym& rec) {
    const uint32_t start = first_unremoved_;
    const uint32_t count = sum_end_ - start;
    const uint8_t rx = row_value(row);
    Pcg32 prng;
    prng.seed(row, count);
    const uint32_t pairs = (count + kPairRate - 1) / kPairRate;
    const size_t at = rec.size();
    rec.resize(at + 2 * (size_t)pairs);
    Term* t = rec.data() + at;
    const FastMod mod(count);
    for (uint32_t i = 0; i < pairs; ++i) {
        const uint32_t e1 = start + mod(prng.next());
        const uint32_t erx = start + mod(prng.next());
        const Segment& s1 = seg_of(e1);
        const Segment& srx = seg_of(erx);
        t[2 * i] = Term{s1.row(e1 + base_ - s1.first), s1.bytes, 1};
        t[2 * i + 1] = Term{srx.row(erx + base_ - srx.first), srx.bytes, rx};
    }
}

void Encoder::light_pairs(uint32_t row, std::vector<uint64_t>& out) {
    const uint32_t start = first_unremoved_;
    const uint32_t count = sum_end_ - start;
    const uint8_t rx = row_value(row);
    Pcg32 prng;
    prng.seed(row, count);
    const uint32_t pairs = (count + kPairRate - 1) / kPairRate;
    out.resize(2 * (size_t)pairs);
    const FastMod mod(count);
    for (uint32_t i = 0; i < pairs; ++i) {
        const uint32_t e1 = start + mod(prng.next());
        const uint32_t erx = start + mod(prng.next());
        out[2 * i] = (uint64_t)(base_ + e1) << 8 | 1u;
        out[2 * i + 1] = (uint64_t)(base_ + erx) << 8 | rx;
    }
    // (a few dozen entries: insertion sort)
    for (size_t i = 1; i < out.size(); ++i) {
        const uint64_t x = out[i];
        size_t j = i;
        while (j > 0 && out[j - 1] > x) {
            out[j] = out[j - 1];
            --j;
        }
        out[j] = x;
    }
}

// Short sum ranges (the usual case with acknowledgements: each Siamese row follows a sum reset)
// are read straight from the packets; long ones through the running lane sums.
bool Encoder::direct_sums() const {
    static const uint32_t direct_max = getenv("TONK_AMD_DIRECT") ? (uint32_t)atoi(getenv("TONK_AMD_DIRECT"))
                                                                  : kDirectMax;
    static const int direct_mode = getenv("TONK_AMD_DIRECT_MODE") ? atoi(getenv("TONK_AMD_DIRECT_MODE")) : 0;
    const uint32_t range = count_ + sum_erased_ - sum_start_;
    const bool fresh = sum_end_ == sum_start_;
    // Direct reads pay per run (a DENSE run's coefficient setup and first row loads); packets
    // added one by one with host copies (the C ABI) are runs of one, where the lane sums' batched
    // single-row reads are far cheaper: direct only while the range's runs average kDirectMinRun.
    bool direct = range <= direct_max && (direct_mode == 0 || fresh || (direct_mode == 2 && range <= 128));
    if (direct && range) direct = (segs_.size() - seg_index_at(sum_abs_start())) * kDirectMinRun <= range;
    return direct;
}

// encode()'s branches without running them: the single packet and Cauchy / parity rows change
// only row counters (and the sum end); a Siamese row also its sum end, unless its lane reads would
// accumulate packets or snapshot a pending scan.
bool Encoder::encode_is_quiet() const {
    if (disabled_ || count_ <= 0 || first_unremoved_ >= kRemoveThreshold) return false;
    const uint32_t un = unacked();
    if (un == 1) return true;
    const uint32_t ub = count_ - sum_start_ + sum_erased_;
    if (sum_end_ <= sum_start_ || ub >= kMaxPackets) return un <= kCauchyThreshold;  // (else a sum reset)
    if (un <= kSumResetThreshold || ub <= kCauchyThreshold) return true;
    if (direct_sums()) return true;
    for (unsigned l = 0; l < kLanes; ++l)
        if ((int32_t)(base_ + count_ - lanes_[l].next_abs) > 0 || !lanes_[l].sums.idle()) return false;
    return true;
}

// Encoder::Encode (SiameseEncoder.cpp:1146-1254)
Result Encoder::encode(RecoveryOut& out) {
    out = RecoveryOut();
    if (disabled_) return kDisabled;
    if (count_ <= 0) return kNeedMoreData;
    if (first_unremoved_ >= kRemoveThreshold) remove_elements();

    const uint32_t un = unacked();
    if (un == 1) return generate_single(out);

    const uint32_t ub = count_ - sum_start_ + sum_erased_;
    if (sum_end_ <= sum_start_ || ub >= kMaxPackets) {
        if (un <= kCauchyThreshold) return generate_cauchy(out);
        reset_sums(first_unremoved_);
    } else if (un <= kSumResetThreshold || ub <= kCauchyThreshold) {
        sum_end_ = sum_start_;
        return generate_cauchy(out);
    }

    const uint32_t row = next_row_;
    if (++next_row_ >= kRowPeriod) next_row_ = 0;

    const uint32_t recovery_bytes = longest_;
    Sym& rec = rec_;
    rec.clear();
    const bool direct = direct_sums();
    if (!direct) {
        TAMD_PROF_SCOPE(kEncDense);
        add_dense(row, recovery_bytes, rec);
    } else {
        sum_end_ = count_;
    }
    {
        TAMD_PROF_SCOPE(kEncLight);
        if (direct) light_pairs(row, pairs_);  // (folded into the dense runs' coefficients)
        else add_light(row, rec);
    }

    RecoveryMeta m;
    m.SumCount = sum_end_ - sum_start_ + sum_erased_;
    m.LDPCCount = un;
    m.ColumnStart = sum_column_start_;
    m.Row = row;
    if (direct) {
        // one op: the dense runs, the LDPC pairs, the store
        out.meta = m;
        out.footer_len = put_recovery_footer(m, out.footer);
        out.data_len = recovery_bytes;
        out.row = ctx_->alloc(recovery_bytes + out.footer_len);
        if (out.row == kNoRow) { disabled_ = true; return kDisabled; }
        if (!defer_dense(row, recovery_bytes, out)) {  // no arena room for its partial sums
            disabled_ = true;
            ctx_->rows.free_deferred(out.row);
            out = RecoveryOut();
            return kDisabled;
        }
        stats_[2]++;
        stats_[3] += out.total();
        return kSuccess;
    }
    // Every term is within recovery_bytes already (lane reads clip to it, packets are at most
    // longest_).  Terms are not merged: the lane snapshots are distinct rows, and a packet the
    // LDPC pairs name twice just becomes two reads (GF(2^8) sums are linear), which costs the
    // device less than a merge costs the host.
    return emit(rec, recovery_bytes, m, out, true);
}

// Encoder::GetStatistics (SiameseEncoder.cpp:1445-1457)
void Encoder::stats(uint64_t* out, unsigned n) {
    if (n > 9) n = 9;
    stats_[8] = ctx_->rows.bytes_in_use();
    for (unsigned i = 0; i < n; ++i) out[i] = stats_[i];
}

} // namespace tamd
