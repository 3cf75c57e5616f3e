// encoder.h -- Siamese encoder control plane (restates SiameseEncoder.h/.cpp of the reference).
//
// State machine identical to the reference: packet window in element order (element % 8 ==
// column % 8), 8 lanes x 3 lazily accumulated running sums, Cauchy/parity rows while few
// packets are in flight and Siamese rows (dense sums + LDPC pairs + RX product) otherwise,
// acknowledgement ingest with NACK-range RTO estimation and retransmit selection.  The only
// difference is that recovery bytes are not computed here: each recovery packet becomes one
// combine op (plus running-sum scans) in the context's device program.
#pragma once

#include <stdio.h>

#include "engine.h"
#include "ring.h"
#include "serial.h"

#include <stdint.h>

namespace tamd {

enum Result {  // siamese.h SiameseResult values
    kSuccess = 0, kInvalidInput = 1, kNeedMoreData = 2, kMaxPacketsReached = 3,
    kDuplicateData = 4, kDisabled = 5
};

struct RecoveryOut {
    RowId row = kNoRow;       // device row: data (data_len bytes) then the footer
    uint32_t data_len = 0;
    uint32_t footer_len = 0;
    uint8_t footer[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    RecoveryMeta meta;
    uint32_t total() const { return data_len + footer_len; }
};

// An original packet as the codec stores it: a device row holding varint(len) || payload.
struct StoredOriginal {
    RowId row = kNoRow;
    uint32_t bytes = 0;         // framed bytes (Buffer.Bytes)
    uint32_t column = 0;
    uint32_t send_msec = 0;     // encoder only (retransmit timing)
    uint32_t off = 0;           // arena offset of `row` (64-B units), cached for program emission
    uint32_t stride = 0;        // off - previous element's off when run > 1
    uint16_t run = 0;           // packets of equal length at a fixed stride ending here (decoder:
                                // received input rows only; 0 for empty and recovered slots)
    uint8_t header_bytes = 0;
    uint8_t owned = 0;          // the codec frees `row` when the packet leaves the window
    void* host = nullptr;       // optional host mirror (C-ABI: siamese_encoder_get/retransmit)
};

typedef void (*HostRelease)(void* host, void* user);

// Whether rows[0..k) are consecutive handles (rows[j] == rows[0] + j).
inline bool consecutive_handles(const RowId* rows, uint32_t k) {
    uint32_t bad = 0;
    for (uint32_t j = 0; j < k; ++j) bad |= rows[j] ^ (rows[0] + j);
    return bad == 0;
}

// A run of consecutive window elements stored as one record ("segment"): equally long framed
// packets whose rows sit at fixed handle and arena strides (row0 + j, off0 + j * stride), none of
// them with a host copy -- a stream's originals added in batches are one segment per stretch
// between events, so adding k of them is O(1) records instead of k.  Any other element (a host
// copy, the C ABI's single adds, placeholders of a restarted window) is a segment of one.
struct Segment {
    uint32_t first = 0;   // absolute element number of the first packet (window element + base)
    uint32_t count = 0;
    RowId row0 = kNoRow;  // kNoRow: placeholders (no packet)
    uint32_t off0 = 0, stride = 0;  // arena offsets in 64-B units; stride 0 when count is 1
    uint32_t bytes = 0;   // framed bytes of every packet (0: placeholder)
    uint32_t column0 = 0; // packet number of the first packet (a segment never wraps the period)
    uint8_t header_bytes = 0;
    uint8_t owned = 0;    // the codec frees the rows when they leave the window
    void* host = nullptr; // count 1 only
    uint32_t end() const { return first + count; }
    RowId row(uint32_t j) const { return row0 == kNoRow ? kNoRow : row0 + j; }
    uint32_t off(uint32_t j) const { return off0 + j * stride; }
};

class Encoder : public FlushClient {
public:
    // Longer direct dense ranges are split (in contexts that ask for it, Context::dense_split):
    // partial sums over chunks of this many packets from the range's start, one combine each
    // (level 1), added by the row's op (level 2), so no single work item walks hundreds of
    // packets (a level's tail).
    static const uint32_t kDenseSplit = 48;
    // Siamese rows whose sum range is at most this many packets read it straight from the packets
    // (defer_dense, and the decoder's Decoder::eliminate_direct); longer ones through the running
    // lane sums (TONK_AMD_DIRECT overrides the encoder's).
    static const uint32_t kDirectMax = 512;
    static const uint32_t kDirectMinRun = 8;  // packets per run the direct reads need on average
    Encoder(Context* ctx, uint32_t row_bytes, HostRelease release = nullptr, void* user = nullptr);
    ~Encoder();

    unsigned remaining_slots() const { return kMaxPackets - count_; }

    // siamese_encoder_add: the caller provides the framed row already written to the arena
    // (a level-0 row: not produced by the pending program).
    // Ownership of `row` (and `host`) passes to the encoder on success unless `borrowed`: a
    // borrowed row stays the caller's (device-resident inputs that outlive the codec).
    Result add(RowId row, uint32_t framed_bytes, uint32_t header_bytes, uint32_t payload_bytes,
               void* host, uint32_t* packet_num, bool borrowed = false);
    // Batched add of k equally long packets (rows[0..k)): the window ends up exactly as after k
    // add() calls.  Returns false, with nothing done, when one of those calls would not succeed.
    // `layout` (nonzero): the caller guarantees rows[j] == rows[0] + j at arena offsets
    // layout >> 32 + j * (layout & 0xffffffff) (a stretch of a session's input rows), so neither
    // is checked nor looked up.
    bool add_run(const RowId* rows, uint32_t k, uint32_t framed_bytes, uint32_t header_bytes,
                 uint32_t payload_bytes, bool borrowed, uint32_t* first_col,
                 uint64_t layout = 0);
    // siamese_encoder_get / _retransmit: the packet as a value (row, lengths, column, host copy)
    Result get(uint32_t packet_num, StoredOriginal* out);
    void remove_before(uint32_t first_kept_column);
    Result acknowledge(const uint8_t* data, uint32_t bytes, uint32_t* next_expected);
    Result retransmit(StoredOriginal* out);
    // siamese_encode.  On success `out.row` is owned by the caller (free it with
    // ctx->rows.free_deferred once nothing reads it).
    Result encode(RecoveryOut& out);
    void stats(uint64_t* out, unsigned n);
    // Encode-ahead (the C ABI's encodes issued before the caller asks, capi.cpp): whether the
    // next encode() would change no state but a Mark's fields -- no removal or sum reset due,
    // and, for a Siamese row over the lane sums, nothing for them to accumulate or scan -- so that
    // encodes run ahead of the caller are taken back exactly by rewind() when another call comes
    // first.  (Rows those encodes allocated stay the caller's to free.)
    struct Mark {
        uint32_t next_row, next_parity_column, next_cauchy_row, sum_end;
        uint64_t recoveries, recovery_bytes;
        bool disabled;
    };
    bool encode_is_quiet() const;
    Mark mark() const {
        return Mark{next_row_, next_parity_column_, next_cauchy_row_, sum_end_, stats_[2], stats_[3], disabled_};
    }
    void rewind(const Mark& m) {
        next_row_ = m.next_row;
        next_parity_column_ = m.next_parity_column;
        next_cauchy_row_ = m.next_cauchy_row;
        sum_end_ = m.sum_end;
        stats_[2] = m.recoveries;
        stats_[3] = m.recovery_bytes;
        disabled_ = m.disabled;
    }
    // Millisecond clock of send times, RTO updates and retransmit decisions (GetTimeMsec in
    // SiameseEncoder.cpp:142, 595, 905).  Default: the monotonic clock; a batch driver may point
    // it at a per-step value or a virtual clock.
    void set_clock(const uint64_t* msec) { clock_ = msec; }

    bool disabled() const { return disabled_; }
    void set_disabled() { disabled_ = true; }
    uint64_t stat(unsigned i) const { return stats_[i]; }

    // FlushClient
    void pre_flush() override;
    void post_flush() override {}

private:
    Context* ctx_;
    uint32_t row_bytes_;
    HostRelease release_;
    void* user_;
    uint64_t stats_[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    bool disabled_ = false;
    const uint64_t* clock_ = nullptr;
    uint64_t now_msec() const;

    // ---- EncoderPacketWindow (SiameseEncoder.h:104-232) ----
    // Elements are stored as segments (Segment, above); per element only its segment number and
    // its send time (retransmit moves single elements' send times).
    struct Slot { uint32_t seg, send_msec; };
    Ring<Slot> win_;
    Ring<Segment> segs_;       // in element order; segs_[i] is segment number seg_base_ + i
    uint32_t seg_base_ = 0;    // number of the segment at segs_[0]
    uint32_t base_ = 0;        // absolute element number of window element 0
    const Segment& seg_of(uint32_t e) const { return segs_[win_[e].seg - seg_base_]; }
    RowId row_of(uint32_t e) const {
        const Segment& s = seg_of(e);
        return s.row(e + base_ - s.first);
    }
    StoredOriginal view(uint32_t e) const;  // element e as a value (get / retransmit)
    // Index in segs_ of the segment holding absolute element `a` (segments below the window are
    // kept while the running sums may still need them, see remove_elements).
    size_t seg_index_at(uint32_t a) const {
        if ((int32_t)(a - base_) >= 0) return win_[a - base_].seg - seg_base_;
        size_t i = 0;
        while (i + 1 < segs_.size() && (int32_t)(segs_[i].end() - a) <= 0) ++i;
        return i;
    }
    uint32_t sum_abs_start() const { return base_ + sum_start_ - sum_erased_; }  // first element of the sums
    // Append k packets (rows[0..k), equally long) at the window end, extending the last segment
    // while the rows continue its strides; `now` is their send time.
    void append(const RowId* rows, uint32_t k, uint32_t framed_bytes, uint32_t header_bytes, uint8_t owned,
                void* host, uint32_t now,
                uint64_t layout = 0);
    void release_segment(const Segment& s, uint32_t from, uint32_t n);  // rows [from, from + n) of s
    void drop_all();                                // release every segment, empty window
    void drop_segments_below(uint32_t drop);        // release segments (parts) below absolute `drop`
    // Send timestamps the placeholder elements of a restarted window read: the reference keeps
    // them in its subwindows' LastSendMsec arrays (SiameseEncoder.h:96), which a window restart
    // (StartNewWindow, SiameseEncoder.cpp:163) does not clear, so an RTT scan that starts on a
    // placeholder (UpdateRTO from a NextRTOColumn before the new window's first packet) sees the
    // previous window's send time at that element, not zero.
    uint32_t placeholder_msec_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t next_column_ = 0, count_ = 0, column_start_ = 0, longest_ = 0;
    uint32_t held_ = 0;  // segments with something to release (owned rows or a host copy)
    uint32_t first_unremoved_ = 0;
    uint32_t sum_start_ = 0, sum_end_ = 0, sum_column_start_ = 0, sum_erased_ = 0;
    // The reference advances each of a lane's three sums lazily on its own; their values only
    // depend on the element they are read at (always Count), so one position per lane suffices.
    struct Lane {
        uint32_t next_abs = 0;  // absolute element number of the lane's next packet to accumulate
        LaneSums sums;
        uint32_t longest = 0;
    } lanes_[kLanes];

    // ---- acknowledgement state (SiameseEncoder.h:239-327) ----
    struct Ack {
        std::vector<uint8_t> data;   // NACK bytes + 8 zero guard bytes
        bool have_data = false;      // reference: Data != nullptr
        uint32_t data_bytes = 0, offset = 0, loss_column = 0, loss_count = 0;
        uint32_t next_expected = 0, next_rto_column = 0;
        bool found_oldest = false;
        uint32_t oldest_column = 0;
        uint32_t rto_msec = 500;
        struct Sample { uint32_t value; uint64_t ts; } max_rtt[3] = {{0, 0}, {0, 0}, {0, 0}};
    } ack_;

    uint32_t next_row_ = 0, next_parity_column_ = 0, next_cauchy_row_ = 0;

    uint32_t to_element(uint32_t column) const { return col_sub(column, column_start_); }
    uint32_t to_column(uint32_t element) const { return col_add(element, column_start_); }
    uint32_t unacked() const { return count_ - first_unremoved_; }
public:
    // Diagnostics (the C ABI watchdog): window and acknowledgement state in one line.
    int debug_state(char* buf, size_t n) const {
        const uint32_t now = (uint32_t)now_msec();
        const uint32_t first = col_sub(ack_.next_expected, column_start_);
        const uint32_t age = first < count_ && first < win_.size() ? now - win_[first].send_msec : 0;
        return snprintf(buf, n,
                        "count=%u first_unremoved=%u next_column=%u column_start=%u ack_next=%u ack_bytes=%u "
                        "rto=%u found_oldest=%d first_age_ms=%u disabled=%d",
                        count_, first_unremoved_, next_column_, column_start_, ack_.next_expected, ack_.data_bytes,
                        ack_.rto_msec, (int)ack_.found_oldest, age, (int)disabled_);
    }
private:
    uint32_t next_lane_element(uint32_t element, uint32_t lane) const {
        uint32_t n = element - (element % kLanes) + lane;
        if (n < element) n += kLanes;
        return n;
    }

    // The first packet of an add (starts a window when it is empty); returns its column.
    uint32_t add_first(RowId row, uint32_t framed_bytes, uint32_t header_bytes, uint32_t payload_bytes, void* host,
                       bool borrowed);
    void start_new_window(uint32_t column);
    void reset_sums(uint32_t element_start);
    void remove_elements();
    LaneSums& get_lane(uint32_t lane, uint32_t element_end);

    bool decode_next_range();
    bool next_loss_column(uint32_t& column);
    void restart_loss_iterator();
    bool on_ack_data(const uint8_t* data, uint32_t bytes);
    void update_rto();
    void rtt_update(uint32_t value, uint64_t now, uint64_t window);
    Result attempt_retransmit(uint32_t e, StoredOriginal* out);

    Result generate_single(RecoveryOut& out);
    Result generate_cauchy(RecoveryOut& out);
    bool direct_sums() const;  // a Siamese row reads its sum range straight from the packets
    void add_dense(uint32_t row, uint32_t recovery_bytes, Sym& rec);
    void add_light(uint32_t row, Sym& rec);
    // The same pair columns as (absolute element << 8 | coefficient), sorted by element.
    void light_pairs(uint32_t row, std::vector<uint64_t>& out);
    std::vector<uint64_t> pairs_;
    Result emit(Sym& terms, uint32_t len, const RecoveryMeta& meta, RecoveryOut& out, bool distinct);
    Sym scratch_, rec_;
    struct Run { RowId row; uint32_t off, stride, count, len, col; };
    std::vector<Run> runs_;
    // Up to three consecutive Cauchy / parity rows of one window generation are emitted together
    // as one op (MULTI runs, program.h): each packet of their windows' union is read once.
    // Windows only move forward (first and end columns never decrease), so the union is each
    // row's runs up to where the next row's window starts.
    struct CauchyTarget {
        RowId row = kNoRow;
        uint32_t used = 0, first_col = 0, end_col = 0, kind = 0, param = 0, flen = 0;
        uint8_t footer[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        std::vector<Run> runs;
    };
    // Union of a group's windows, in packets (within the 11-bit run indices of TARGETS).  Round 3
    // kept rows over windows of 32 packets or more alone (pure combines the executor may share
    // across a workgroup in small launches); with acknowledgements every 64 packets and f = 4 %
    // (configs[2]) consecutive Cauchy windows of ~50 packets overlap by half, and grouping them
    // reads 27 % fewer window rows (cp_bench reads: 5998 -> 4366 per 4096 originals).
    static const uint32_t kGroupSpan = 160;
    CauchyTarget grp_[3];
    uint32_t grp_n_ = 0, grp_gen_ = 0, window_gen_ = 0;
    std::vector<Run> grp_union_;
    void emit_cauchy_group();

    // Up to three consecutive direct Siamese rows of one sum range are emitted together as one
    // op per chunk (DENSE runs with targets, program.h).  Between two sum resets every row's range
    // starts at the same element and ends at the window end of its encode, so the ranges are
    // nested and the last row's runs are their union: each packet is read once for the group
    // instead of once per row (a packet was read by ~4 rows on the headline workload).
    struct DenseRun { uint32_t off, stride, count, len, col, e0; };  // e0: absolute first element
    struct DenseTarget {
        RowId row = kNoRow;
        uint64_t ops = 0;            // lane opcodes, 6 bits each
        uint32_t hi = 0, flen = 0;   // absolute end of the range; footer bytes
        uint8_t rx = 0;
        uint8_t footer[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        std::vector<uint64_t> pairs; // LDPC pair columns inside its runs: (element - lo) << 8 | coef
        Sym loose;                   // the others, as rows
        std::vector<RowId> parts;    // partial sums, one per chunk (ranges over one chunk: none)
    };
    // Packets x rows one group op may take per chunk (TONK_AMD_DENSE_WORK overrides): a chunk
    // of 192 packets (kDenseSplit) is one row's work; its items are the level's longest.
    static const uint32_t kDenseGroupWork = 144;
    DenseTarget dgrp_[3];
    uint32_t dgrp_n_ = 0, dgrp_lo_ = 0, dgrp_len_ = 0, dgrp_gen_ = 0;
    std::vector<DenseRun> dgrp_runs_;  // the runs of [lo, hi) of the group's last row
    // Queue `out.row` (allocated, footer set) with the group; false: no arena room for its
    // partial sums (the codec is disabled).
    bool defer_dense(uint32_t row, uint32_t recovery_bytes, const RecoveryOut& out);
    void emit_dense_group();
};

uint64_t time_msec();
void set_clock_source(uint64_t (*fn)());  // test hook: replaces the clock time_msec() reads
inline uint64_t Encoder::now_msec() const { return clock_ ? *clock_ : time_msec(); }

} // namespace tamd
