// Minimal Optional (reference include/madrona/optional.hpp:17-150) for the
// graph API's optional parent node; trivially copyable payloads only.
#pragma once

#include <madrona/hd.hpp>

#include <type_traits>
#include <utility>

namespace madrona {

template <typename T>
class Optional {
    static_assert(std::is_trivially_copyable_v<T>, "Optional<T> holds trivially copyable T");
public:
    static constexpr MW_INLINE Optional none() { return Optional(); }
    template <typename... Args>
    static constexpr MW_INLINE Optional make(Args &&...args)
    {
        Optional o;
        o.value_ = T { std::forward<Args>(args)... };
        o.has_ = true;
        return o;
    }
    constexpr MW_INLINE Optional() : value_ {}, has_(false) {}
    constexpr MW_INLINE Optional(const T &v) : value_(v), has_(true) {}

    constexpr MW_INLINE bool has_value() const { return has_; }
    constexpr MW_INLINE explicit operator bool() const { return has_; }
    constexpr MW_INLINE const T &operator*() const { return value_; }
    constexpr MW_INLINE T &operator*() { return value_; }
    constexpr MW_INLINE const T *operator->() const { return &value_; }
    constexpr MW_INLINE T *operator->() { return &value_; }

private:
    T value_;
    bool has_;
};

}
