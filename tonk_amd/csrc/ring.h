// ring.h -- random-access window with cheap removal from the front (window elements).
#pragma once
#include <stddef.h>
#include <vector>

namespace tamd {

template <class T>
class Ring {
public:
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    T& back() { return buf_[(head_ + n_ - 1) & mask_]; }
    const T& back() const { return buf_[(head_ + n_ - 1) & mask_]; }
    T& front() { return buf_[head_]; }
    T& operator[](size_t i) { return buf_[(head_ + i) & mask_]; }
    const T& operator[](size_t i) const { return buf_[(head_ + i) & mask_]; }
    void push_back(const T& v) {
        if (n_ == buf_.size()) grow();
        buf_[(head_ + n_) & mask_] = v;
        ++n_;
    }
    // Bulk append: make room for k more, fill slot(n + j) for j < k, then commit(k).
    void reserve_more(size_t k) {
        while (n_ + k > buf_.size()) grow();
    }
    T* slot_base() { return buf_.data(); }
    size_t slot_index(size_t i) const { return (head_ + i) & mask_; }
    size_t slot_mask() const { return mask_; }
    void commit(size_t k) { n_ += k; }
    // Append a slot to fill in place (no temporary: a struct built in narrow fields and then
    // copied with wide loads stalls on store forwarding).
    T& push_slot() {
        if (n_ == buf_.size()) grow();
        return buf_[(head_ + n_++) & mask_];
    }
    void pop_front(size_t k) {
        if (k > n_) k = n_;
        // (popped slots keep stale contents: push_back and push_slot rewrite every field)
        head_ = (head_ + k) & mask_;
        n_ -= k;
    }
    void clear() { pop_front(n_); head_ = 0; }

private:
    std::vector<T> buf_;
    size_t head_ = 0, n_ = 0, mask_ = 0;
    void grow() {
        const size_t cap = buf_.empty() ? 64 : buf_.size() * 2;
        std::vector<T> nb(cap);
        for (size_t i = 0; i < n_; ++i) nb[i] = (*this)[i];
        buf_.swap(nb);
        head_ = 0;
        mask_ = cap - 1;
    }
};

} // namespace tamd
