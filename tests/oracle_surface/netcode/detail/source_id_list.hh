// tests/oracle_surface (tests only): a sorted set of source ids (the reference's
// detail/source_id_list.hh is a boost flat_set<uint32_t>).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <initializer_list>
#include <utility>
#include <vector>

namespace ntc {
namespace detail {

class source_id_list
{
public:
  using value_type = std::uint32_t;
  using size_type = std::size_t;
  using iterator = std::vector<std::uint32_t>::iterator;
  using const_iterator = std::vector<std::uint32_t>::const_iterator;
  using reverse_iterator = std::vector<std::uint32_t>::reverse_iterator;
  using const_reverse_iterator = std::vector<std::uint32_t>::const_reverse_iterator;

  source_id_list() = default;
  source_id_list(std::initializer_list<std::uint32_t> ids) : v_(ids) { normalise(); }
  template <typename It> source_id_list(It first, It last) : v_(first, last) { normalise(); }

  std::pair<iterator, bool> insert(std::uint32_t x)
  {
    auto it = std::lower_bound(v_.begin(), v_.end(), x);
    if (it != v_.end() && *it == x) return {it, false};
    return {v_.insert(it, x), true};
  }
  iterator insert(const_iterator, std::uint32_t x) { return insert(x).first; }   // hint ignored
  iterator erase(const_iterator it) { return v_.erase(it); }
  size_type erase(std::uint32_t x)
  {
    auto it = find(x);
    if (it == v_.end()) return 0;
    v_.erase(it);
    return 1;
  }
  iterator find(std::uint32_t x)
  {
    auto it = std::lower_bound(v_.begin(), v_.end(), x);
    return it != v_.end() && *it == x ? it : v_.end();
  }
  const_iterator find(std::uint32_t x) const
  {
    auto it = std::lower_bound(v_.begin(), v_.end(), x);
    return it != v_.end() && *it == x ? it : v_.end();
  }
  size_type count(std::uint32_t x) const { return find(x) != v_.end() ? 1 : 0; }

  iterator begin() noexcept { return v_.begin(); }
  const_iterator begin() const noexcept { return v_.begin(); }
  const_iterator cbegin() const noexcept { return v_.cbegin(); }
  iterator end() noexcept { return v_.end(); }
  const_iterator end() const noexcept { return v_.end(); }
  const_iterator cend() const noexcept { return v_.cend(); }
  reverse_iterator rbegin() noexcept { return v_.rbegin(); }
  const_reverse_iterator rbegin() const noexcept { return v_.rbegin(); }
  reverse_iterator rend() noexcept { return v_.rend(); }
  const_reverse_iterator rend() const noexcept { return v_.rend(); }

  size_type size() const noexcept { return v_.size(); }
  bool empty() const noexcept { return v_.empty(); }
  void clear() noexcept { v_.clear(); }
  void reserve(size_type n) { v_.reserve(n); }
  const std::uint32_t* data() const noexcept { return v_.data(); }

  friend bool operator==(const source_id_list& a, const source_id_list& b) { return a.v_ == b.v_; }
  friend bool operator!=(const source_id_list& a, const source_id_list& b) { return a.v_ != b.v_; }

private:
  void normalise()
  {
    std::sort(v_.begin(), v_.end());
    v_.erase(std::unique(v_.begin(), v_.end()), v_.end());
  }

  std::vector<std::uint32_t> v_;
};

// begin(ids) / end(ids) by ADL, as for the reference's boost container (std:: template arguments)
inline source_id_list::iterator begin(source_id_list& s) noexcept { return s.begin(); }
inline source_id_list::const_iterator begin(const source_id_list& s) noexcept { return s.begin(); }
inline source_id_list::iterator end(source_id_list& s) noexcept { return s.end(); }
inline source_id_list::const_iterator end(const source_id_list& s) noexcept { return s.end(); }

}  // namespace detail
}  // namespace ntc
