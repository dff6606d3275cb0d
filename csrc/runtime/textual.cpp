// Native `.moose` textual parser (see textual.h).
#include "textual.h"

#include <array>
#include <climits>
#include <cstring>
#include <system_error>
#include <thread>

namespace moosert {
namespace {

inline bool is_ident(char c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ||
         c == '_';
}
inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
inline bool is_hex(char c) {
  return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}
inline int hexval(char c) {
  if (is_digit(c)) return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  return c - 'A' + 10;
}

class Cursor {
 public:
  Cursor(std::string_view s, size_t base_line) : s_(s), line_base_(base_line) {}

  void ws() {
    while (i_ < s_.size()) {
      char c = s_[i_];
      if (c == ' ' || c == '\t' || c == '\n' || c == '\r') {
        ++i_;
      } else if (c == '/' && i_ + 1 < s_.size() && s_[i_ + 1] == '/') {
        while (i_ < s_.size() && s_[i_] != '\n' && s_[i_] != '\r') ++i_;
      } else {
        break;
      }
    }
  }
  bool at_end() {
    ws();
    return i_ >= s_.size();
  }
  bool peek(std::string_view lit) {
    ws();
    return s_.substr(i_, lit.size()) == lit;
  }
  bool eat(std::string_view lit) {
    if (peek(lit)) {
      i_ += lit.size();
      return true;
    }
    return false;
  }
  void expect(std::string_view lit) {
    if (!eat(lit)) fail("expected '" + std::string(lit) + "'");
  }
  std::string_view ident(const char* what) {
    ws();
    size_t j = i_;
    while (j < s_.size() && is_ident(s_[j])) ++j;
    if (j == i_) fail(std::string("expected ") + what);
    auto r = s_.substr(i_, j - i_);
    i_ = j;
    return r;
  }
  // [-+]?(\d+\.\d*|\.\d+|\d+)([eE][-+]?\d+)? | [-+]?inf | NaN
  Num number() {
    ws();
    size_t j = i_;
    if (j < s_.size() && (s_[j] == '-' || s_[j] == '+')) ++j;
    if (s_.substr(j, 3) == "inf") {
      Num n{s_.substr(i_, j + 3 - i_), true};
      i_ = j + 3;
      return n;
    }
    if (j == i_ && s_.substr(j, 3) == "NaN") {
      i_ = j + 3;
      return Num{s_.substr(j - 0, 3), true};
    }
    size_t d0 = j;
    while (j < s_.size() && is_digit(s_[j])) ++j;
    bool flt = false;
    bool digits = j > d0;
    if (j < s_.size() && s_[j] == '.') {
      size_t k = j + 1;
      while (k < s_.size() && is_digit(s_[k])) ++k;
      if (digits || k > j + 1) {
        flt = true;
        digits = true;
        j = k;
      }
    }
    if (!digits) fail("expected number");
    if (j < s_.size() && (s_[j] == 'e' || s_[j] == 'E')) {
      size_t k = j + 1;
      if (k < s_.size() && (s_[k] == '-' || s_[k] == '+')) ++k;
      size_t e0 = k;
      while (k < s_.size() && is_digit(s_[k])) ++k;
      if (k > e0) {
        flt = true;
        j = k;
      }
    }
    Num n{s_.substr(i_, j - i_), flt};
    i_ = j;
    return n;
  }
  int64_t integer() {
    Num n = number();
    if (n.is_float) fail("expected integer");
    return std::stoll(std::string(n.tok));
  }
  std::string string_lit() {
    ws();
    if (i_ >= s_.size() || s_[i_] != '"') fail("expected string");
    std::string out;
    size_t j = i_ + 1;
    while (j < s_.size() && s_[j] != '"') {
      if (s_[j] == '\\' && j + 1 < s_.size()) {
        out.push_back(s_[j + 1]);
        j += 2;
      } else {
        out.push_back(s_[j++]);
      }
    }
    if (j >= s_.size()) fail("unterminated string");
    i_ = j + 1;
    return out;
  }
  std::string_view hex_run() {
    ws();
    size_t j = i_;
    while (j < s_.size() && is_hex(s_[j])) ++j;
    if (j == i_) fail("expected hex");
    auto r = s_.substr(i_, j - i_);
    i_ = j;
    return r;
  }
  // [A-Za-z0-9]+(<[^>]*>)?
  std::string_view type() {
    ws();
    size_t j = i_;
    while (j < s_.size() && (is_ident(s_[j]) && s_[j] != '_')) ++j;
    if (j == i_) fail("expected a type");
    if (j < s_.size() && s_[j] == '<') {
      size_t k = s_.find('>', j);
      if (k == std::string_view::npos) fail("unterminated type parameter");
      j = k + 1;
    }
    auto r = s_.substr(i_, j - i_);
    i_ = j;
    return r;
  }

  // nested list of numbers -> flat + shape (rectangular)
  void nested(std::vector<Num>& flat, std::vector<int64_t>& shape) {
    shape.clear();
    std::vector<int64_t> counts;
    nested_rec(flat, shape, 0);
  }

  [[noreturn]] void fail(const std::string& msg) {
    size_t line = line_base_ + 1;
    for (size_t k = 0; k < i_ && k < s_.size(); ++k)
      if (s_[k] == '\n') ++line;
    size_t e = s_.find('\n', i_);
    auto snip = s_.substr(i_, std::min<size_t>(60, (e == std::string_view::npos ? s_.size() : e) - i_));
    throw ParseError("line " + std::to_string(line) + ": " + msg + " at '" + std::string(snip) +
                     "'");
  }

 private:
  void nested_rec(std::vector<Num>& flat, std::vector<int64_t>& shape, size_t depth) {
    if (eat("[")) {
      int64_t n = 0;
      if (!eat("]")) {
        while (true) {
          nested_rec(flat, shape, depth + 1);
          ++n;
          if (eat("]")) break;
          expect(",");
        }
      }
      if (shape.size() <= depth) {
        shape.resize(depth + 1, -1);
      }
      if (shape[depth] == -1) {
        shape[depth] = n;
      } else if (shape[depth] != n) {
        fail("ragged tensor literal");
      }
      return;
    }
    flat.push_back(number());
  }

  std::string_view s_;
  size_t i_ = 0;
  size_t line_base_;
};

const std::string_view kTensorConsts[] = {
    "HostFloat32Tensor", "HostFloat64Tensor", "HostInt8Tensor",   "HostInt16Tensor",
    "HostInt32Tensor",   "HostInt64Tensor",   "HostUint8Tensor",  "HostUint16Tensor",
    "HostUint32Tensor",  "HostUint64Tensor",  "HostRing64Tensor", "HostRing128Tensor",
    "HostBitTensor"};

bool is_tensor_const(std::string_view k) {
  for (auto t : kTensorConsts)
    if (t == k) return true;
  return false;
}

void parse_constant_literal(Cursor& c, std::string_view kind, Value& v) {
  v.tag = Value::Const;
  c.expect("(");
  if (is_tensor_const(kind)) {
    v.ckind = std::string(kind);
    v.const_is_tensor = true;
    c.nested(v.nums, v.shape);
  } else if (kind == "HostShape") {
    v.ckind = "HostShape";
    std::vector<int64_t> sh;
    c.nested(v.nums, sh);
  } else if (kind == "HostString" || kind == "String") {
    v.ckind = "HostString";
    v.text = c.string_lit();
  } else if (kind == "HostSeed" || kind == "HostPrfKey" || kind == "Seed" || kind == "PrfKey") {
    v.ckind = (kind == "Seed") ? "HostSeed" : (kind == "PrfKey") ? "HostPrfKey" : std::string(kind);
    if (c.peek("[")) {
      std::vector<Num> raw;
      std::vector<int64_t> sh;
      c.nested(raw, sh);
      for (auto& n : raw) v.bytes.push_back(static_cast<uint8_t>(std::stoi(std::string(n.tok))));
    } else {
      auto h = c.hex_run();
      if (h.size() % 2) c.fail("odd-length hex");
      for (size_t k = 0; k < h.size(); k += 2)
        v.bytes.push_back(static_cast<uint8_t>(hexval(h[k]) * 16 + hexval(h[k + 1])));
    }
  } else if (kind == "Ring64" || kind == "Ring128" || kind == "Bit") {
    v.ckind = std::string(kind);
    Num n = c.number();
    if (n.is_float) c.fail("expected integer");
    v.nums.push_back(n);
  } else if (kind == "Float32" || kind == "Float64") {
    v.ckind = std::string(kind);
    v.nums.push_back(c.number());
  } else if (kind == "Fixed") {
    v.ckind = "Fixed";
    v.nums.push_back(c.number());
    c.expect(",");
    v.nums.push_back(c.number());
    if (c.peek(",")) {
      c.expect(",");
      v.nums.push_back(c.number());
    } else {  // the reference's Fixed(value, precision): integral precision 0
      v.nums.insert(v.nums.begin() + 1, Num{std::string_view("0"), false});
    }
  } else {
    c.fail("unknown constant kind " + std::string(kind));
  }
  c.expect(")");
}

void parse_key(Cursor& c, Value& v) {
  v.tag = Value::Key;
  if (c.peek("[")) {
    std::vector<Num> raw;
    std::vector<int64_t> sh;
    c.nested(raw, sh);
    for (auto& n : raw) v.bytes.push_back(static_cast<uint8_t>(std::stoi(std::string(n.tok))));
    return;
  }
  auto h = c.hex_run();
  std::string padded(h);
  if (padded.size() < 32) padded.insert(0, 32 - padded.size(), '0');
  if (padded.size() % 2) padded.insert(0, 1, '0');
  for (size_t k = 0; k < padded.size(); k += 2)
    v.bytes.push_back(static_cast<uint8_t>(hexval(padded[k]) * 16 + hexval(padded[k + 1])));
}

void parse_slice(Cursor& c, Value& v) {
  v.tag = Value::Slice;
  auto one = [&]() {
    std::array<int64_t, 3> s{0, INT64_MIN, INT64_MIN};
    c.expect("{");
    while (!c.eat("}")) {
      auto k = c.ident("slice field");
      c.expect("=");
      int64_t val = c.eat("None") ? INT64_MIN : c.integer();
      if (k == "start") {
        s[0] = val == INT64_MIN ? 0 : val;
      } else if (k == "end") {
        s[1] = val;
      } else if (k == "step") {
        s[2] = val;
      } else {
        c.fail("unknown slice field");
      }
      c.eat(",");
    }
    v.slices.push_back(s);
  };
  if (c.eat("[")) {
    v.slice_list = true;
    while (!c.eat("]")) {
      one();
      c.eat(",");
    }
    return;
  }
  one();
}

void parse_value(Cursor& c, AttrKind k, Value& v) {
  switch (k) {
    case AttrKind::Key:
      parse_key(c, v);
      return;
    case AttrKind::Str:
      v.tag = Value::Str;
      v.text = c.string_lit();
      return;
    case AttrKind::Bool: {
      v.tag = Value::Bool;
      v.b = c.ident("bool") == "true";
      return;
    }
    case AttrKind::Int:
    case AttrKind::OptInt:
      if (c.eat("None")) {
        v.tag = Value::None;
        return;
      }
      v.tag = Value::Int;
      v.num = c.number();
      if (v.num.is_float) c.fail("expected integer");
      return;
    case AttrKind::Ints:
    case AttrKind::OptInts: {
      if (k == AttrKind::OptInts && c.eat("None")) {
        v.tag = Value::None;
        return;
      }
      v.tag = Value::Ints;
      std::vector<int64_t> sh;
      c.nested(v.nums, sh);
      return;
    }
    case AttrKind::Const: {
      if (c.peek("\"")) {
        v.tag = Value::Const;
        v.ckind = "HostString";
        v.text = c.string_lit();
        return;
      }
      auto kind = c.ident("constant kind");
      parse_constant_literal(c, kind, v);
      return;
    }
    case AttrKind::Slice:
      parse_slice(c, v);
      return;
  }
}

OpRecord parse_operation(Cursor& c, const Schema& schema) {
  OpRecord op;
  op.name = c.ident("identifier");
  c.expect("=");
  std::string_view kind = c.ident("operator name");
  auto al = schema.aliases.find(kind);
  op.kind = al != schema.aliases.end() ? al->second : std::string(kind);
  auto it = schema.ops.find(op.kind);
  if (it == schema.ops.end()) c.fail("unknown operator " + op.kind);
  const auto& attrs = it->second;
  std::vector<bool> seen(attrs.size(), false);
  std::vector<Value> vals(attrs.size());
  if (c.eat("{")) {
    while (!c.eat("}")) {
      auto an = c.ident("attribute name");
      c.expect("=");
      size_t idx = attrs.size();
      for (size_t k = 0; k < attrs.size(); ++k)
        if (attrs[k].first == an) idx = k;
      if (idx == attrs.size())
        c.fail("unknown attribute " + std::string(an) + " for " + op.kind);
      parse_value(c, attrs[idx].second, vals[idx]);
      seen[idx] = true;
      c.eat(",");
    }
  }
  for (size_t k = 0; k < attrs.size(); ++k) {
    if (!seen[k]) {
      auto ak = attrs[k].second;
      if (ak == AttrKind::OptInt || ak == AttrKind::OptInts) {
        vals[k].tag = Value::None;
      } else if ((op.kind == "Output" && attrs[k].first == "tag") ||
                 (op.kind == "Input" && attrs[k].first == "arg_name")) {
        vals[k].tag = Value::Str;  // older files omit these (examples/test.moose)
        vals[k].text = std::string(op.name);
      } else {
        c.fail("missing attribute " + attrs[k].first + " for " + op.kind);
      }
    }
    op.attrs.emplace_back(attrs[k].first, std::move(vals[k]));
  }
  if (c.eat(":")) {
    op.has_sig = true;
    if (c.eat("[")) {
      op.variadic = true;
      op.sig_args.push_back(c.type());
      c.expect("]");
      c.expect("->");
      op.sig_ret = c.type();
    } else {
      c.expect("(");
      if (!c.eat(")")) {
        while (true) {
          op.sig_args.push_back(c.type());
          if (c.eat(")")) break;
          c.expect(",");
        }
      }
      c.expect("->");
      op.sig_ret = c.type();
    }
  } else {
    auto d = schema.default_return.find(op.kind);
    if (d == schema.default_return.end()) c.fail("expected a type signature");
    op.sig_ret_default = d->second;
  }
  if (c.eat("(")) {
    if (!c.eat(")")) {
      while (true) {
        op.inputs.push_back(c.ident("input name"));
        if (c.eat(")")) break;
        c.expect(",");
      }
    }
  }
  c.expect("@");
  op.plc_kind = c.ident("placement kind");
  c.expect("(");
  while (true) {
    op.owners.push_back(c.ident("role"));
    if (c.eat(")")) break;
    c.expect(",");
  }
  size_t want = op.plc_kind == "Host"                                          ? 1
                : (op.plc_kind == "Replicated" || op.plc_kind == "Mirrored3") ? 3
                : op.plc_kind == "Additive"                                    ? 2
                                                                               : 0;
  if (want == 0) c.fail("unknown placement kind " + std::string(op.plc_kind));
  if (op.owners.size() != want)
    c.fail(std::string(op.plc_kind) + " placement expects " + std::to_string(want) + " owners");
  return op;
}

std::vector<OpRecord> parse_chunk(std::string_view src, size_t line_base, const Schema& schema) {
  Cursor c(src, line_base);
  std::vector<OpRecord> ops;
  while (!c.at_end()) ops.push_back(parse_operation(c, schema));
  return ops;
}

}  // namespace

std::vector<OpRecord> parse_computation(std::string_view src, const Schema& schema,
                                        int threads) {
  if (threads <= 1 || src.size() < (1u << 16)) return parse_chunk(src, 0, schema);
  // split at line breaks into `threads` chunks (reference parsing.rs:83-117)
  std::vector<std::pair<size_t, size_t>> parts;
  size_t step = src.size() / threads, left = 0;
  for (int t = 0; t < threads && left < src.size(); ++t) {
    size_t right = std::min(src.size(), left + step);
    if (t == threads - 1) right = src.size();
    size_t nl = src.find('\n', right);
    right = nl == std::string_view::npos ? src.size() : nl + 1;
    if (right > left) parts.emplace_back(left, right);
    left = right;
  }
  if (left < src.size()) parts.emplace_back(left, src.size());
  // line offsets of each chunk, for error messages
  std::vector<size_t> line_base(parts.size(), 0);
  for (size_t p = 1; p < parts.size(); ++p) {
    size_t n = 0;
    for (size_t k = parts[p - 1].first; k < parts[p - 1].second; ++k) n += src[k] == '\n';
    line_base[p] = line_base[p - 1] + n;
  }
  std::vector<std::vector<OpRecord>> results(parts.size());
  std::vector<std::string> errors(parts.size());
  auto parse = [&](size_t p) {
    try {
      results[p] = parse_chunk(src.substr(parts[p].first, parts[p].second - parts[p].first),
                               line_base[p], schema);
    } catch (const std::exception& e) {
      errors[p] = e.what();
    }
  };
  std::vector<std::thread> pool;
  size_t started = 0;
  try {
    for (; started < parts.size(); ++started) pool.emplace_back(parse, started);
  } catch (const std::system_error&) {
    // no more threads (the process's limit under load): the rest parse on this thread
    // (a joinable std::thread must never be destroyed)
    for (size_t p = started; p < parts.size(); ++p) parse(p);
  }
  for (auto& th : pool) th.join();
  for (auto& e : errors)
    if (!e.empty()) throw ParseError(e);
  std::vector<OpRecord> out;
  size_t total = 0;
  for (auto& r : results) total += r.size();
  out.reserve(total);
  for (auto& r : results)
    for (auto& op : r) out.push_back(std::move(op));
  return out;
}

}  // namespace moosert
