// netcode/detail/source_id_list.hh -- the sorted set of source ids a repair covers or an ack
// acknowledges (reference netcode/detail/source_id_list.hh: a flat set of u32).  Kept as a sorted
// contiguous vector: id lists are short, iterated in order and written run-length coded
// (packetizer.hh:263-309), and tests index them with random-access iterators.
#pragma once

#include <algorithm>
#include <cstdint>
#include <initializer_list>
#include <vector>

namespace ntc {
namespace detail {

class source_id_list
{
  using storage = std::vector<std::uint32_t>;

public:
  using value_type = std::uint32_t;
  using key_type = std::uint32_t;
  using size_type = storage::size_type;
  using iterator = storage::const_iterator;          // elements are keys: never writable
  using const_iterator = storage::const_iterator;
  using const_reverse_iterator = storage::const_reverse_iterator;
  using reverse_iterator = const_reverse_iterator;

  source_id_list() = default;
  source_id_list(std::initializer_list<std::uint32_t> ids) { insert(ids.begin(), ids.end()); }
  template <typename It>
  source_id_list(It first, It last) { insert(first, last); }

  // Inserts an id; (position, whether it was new).
  std::pair<iterator, bool> insert(std::uint32_t id)
  {
    auto pos = std::lower_bound(v_.begin(), v_.end(), id);
    if (pos != v_.end() && *pos == id) return {pos, false};
    return {v_.insert(pos, id), true};
  }
  iterator insert(const_iterator /*hint*/, std::uint32_t id) { return insert(id).first; }
  template <typename It>
  void insert(It first, It last)
  {
    for (; first != last; ++first) insert(static_cast<std::uint32_t>(*first));
  }
  template <typename... Args>
  std::pair<iterator, bool> emplace(Args&&... args) { return insert(std::uint32_t(args...)); }

  size_type erase(std::uint32_t id)
  {
    auto pos = find(id);
    if (pos == v_.end()) return 0;
    v_.erase(pos);
    return 1;
  }
  iterator erase(const_iterator pos) { return v_.erase(pos); }
  iterator erase(const_iterator first, const_iterator last) { return v_.erase(first, last); }
  void clear() noexcept { v_.clear(); }
  void reserve(size_type n) { v_.reserve(n); }

  const_iterator find(std::uint32_t id) const
  {
    auto pos = std::lower_bound(v_.begin(), v_.end(), id);
    return (pos != v_.end() && *pos == id) ? pos : v_.end();
  }
  size_type count(std::uint32_t id) const { return find(id) == v_.end() ? 0 : 1; }
  const_iterator lower_bound(std::uint32_t id) const { return std::lower_bound(v_.begin(), v_.end(), id); }
  const_iterator upper_bound(std::uint32_t id) const { return std::upper_bound(v_.begin(), v_.end(), id); }

  const_iterator begin() const noexcept { return v_.begin(); }
  const_iterator end() const noexcept { return v_.end(); }
  const_iterator cbegin() const noexcept { return v_.cbegin(); }
  const_iterator cend() const noexcept { return v_.cend(); }
  const_reverse_iterator rbegin() const noexcept { return v_.rbegin(); }
  const_reverse_iterator rend() const noexcept { return v_.rend(); }
  std::uint32_t front() const { return v_.front(); }
  std::uint32_t back() const { return v_.back(); }
  std::uint32_t operator[](size_type i) const { return v_[i]; }
  size_type size() const noexcept { return v_.size(); }
  bool empty() const noexcept { return v_.empty(); }

  friend bool operator==(const source_id_list& a, const source_id_list& b) { return a.v_ == b.v_; }
  friend bool operator!=(const source_id_list& a, const source_id_list& b) { return a.v_ != b.v_; }

private:
  storage v_;
};

// Free begin / end found by argument-dependent lookup (`begin(ids)` in the reference's tests).
inline source_id_list::const_iterator begin(const source_id_list& l) noexcept { return l.begin(); }
inline source_id_list::const_iterator end(const source_id_list& l) noexcept { return l.end(); }

}  // namespace detail
}  // namespace ntc
