// Native parser for the textual `.moose` computation format.
//
// Parity: reference moose/src/textual/parsing.rs (verbose parser :61, fast parser :73,
// parallel_parse_computation :83-117 which splits the source at line breaks and parses
// the chunks on a rayon pool; placements :190; constant literals :608).  Here the
// chunks are parsed on std::threads into flat C++ records that hold string_views into
// the source; the Python binding turns them into IR objects on the calling thread.
#pragma once

#include <array>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace moosert {

// Attribute kinds of the operator schema (moose_amd/ir/operators.py).
enum class AttrKind : uint8_t { Int, OptInt, Ints, OptInts, Bool, Str, Key, Const, Slice };

struct Schema {
  // operator -> ordered (attribute, kind)
  std::map<std::string, std::vector<std::pair<std::string, AttrKind>>, std::less<>> ops;
  std::map<std::string, std::string, std::less<>> aliases;         // deprecated names
  std::map<std::string, std::string, std::less<>> default_return;  // DeriveSeed -> HostSeed
};

// A parsed literal number, kept as its source token (converted exactly on the Python
// side: ints of any width, floats via strtod).
struct Num {
  std::string_view tok;
  bool is_float;
};

struct Value {
  enum Tag : uint8_t {
    None,
    Int,      // num
    Bool,     // b
    Str,      // text (already unescaped)
    Ints,     // nums
    Key,      // bytes (16)
    Const,    // ckind + (tensor: nums + shape | scalar: nums[0] | str: text | bytes)
    Slice,    // slices
  } tag = None;
  Num num{};
  bool b = false;
  std::string text;
  std::string ckind;
  std::vector<Num> nums;
  std::vector<int64_t> shape;
  std::vector<uint8_t> bytes;
  bool const_is_tensor = false;
  // (start, end, step); INT64_MIN marks None
  std::vector<std::array<int64_t, 3>> slices;
  bool slice_list = false;
};

struct OpRecord {
  std::string_view name;
  std::string kind;  // canonical (alias resolved)
  std::vector<std::pair<std::string, Value>> attrs;  // schema order
  std::vector<std::string_view> sig_args;
  std::string_view sig_ret;
  std::string sig_ret_default;  // used when the signature is omitted
  bool has_sig = false;
  bool variadic = false;
  std::vector<std::string_view> inputs;
  std::string_view plc_kind;
  std::vector<std::string_view> owners;
};

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Parse `src` (must outlive the records).  threads <= 1 parses sequentially.
std::vector<OpRecord> parse_computation(std::string_view src, const Schema& schema,
                                        int threads);

}  // namespace moosert
