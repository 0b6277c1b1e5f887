// mdg_jcampdx.cpp -- native decoder of JCAMP-DX data blocks (host code; §8 row f4).
//
// Restates JcampDx::decode_asdf / decode_affn of the reference
// (metabodecon/src/spectrum/formats/jcampdx.rs:892-1091) for ASCII data blocks: the
// same six rewriting passes, each a scan with the match semantics of its regex
// (jcampdx.rs:481-488; leftmost-first, greedy, as the `regex` crate reports them),
// applied in the same order, the DIF/DUP pair repeated until neither matches, then
// the AFFN split (every line minus its first token, f64 FromStr, times the factor).
// So the values are the reference's, including its reading of a DUP after a DIF
// (the decoded value repeated, not the difference).
//
// Any input this restatement does not take on -- a non-ASCII byte (Rust's \s and \d
// are Unicode classes), a token the reference's parse would reject (it panics on a
// bad DIF/DUP base, reports MalformedData on a bad value) -- returns
// MDG_INVALID_ARGUMENT, and the Python reader (metabodecon/_jcampdx.py, the regex
// restatement) decodes that block and raises the reference's error.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mdgpu.h"

namespace {

inline bool is_ws(char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }  // ASCII White_Space
inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
inline bool is_asdf(char c) {  // [@%A-Za-z+-]
    return c == '@' || c == '%' || c == '+' || c == '-' || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z');
}
inline bool is_dif(char c) { return c == '%' || (c >= 'J' && c <= 'R') || (c >= 'j' && c <= 'r'); }
inline bool is_dup(char c) { return (c >= 'S' && c <= 'Z') || c == 's'; }
inline bool is_sqz(char c) { return c == '@' || (c >= 'A' && c <= 'I') || (c >= 'a' && c <= 'i'); }

struct Fail {};

// i64::from_str: optional sign, one or more ASCII digits, no overflow
int64_t parse_i64(const std::string& s) {
    size_t i = 0;
    bool neg = false;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
    if (i == s.size()) throw Fail{};
    __int128 v = 0;
    for (; i < s.size(); ++i) {
        if (!is_digit(s[i])) throw Fail{};
        v = v * 10 + (s[i] - '0');
        if (v > ((__int128)1 << 63)) throw Fail{};
    }
    if (neg) v = -v;
    if (v > INT64_MAX || v < INT64_MIN) throw Fail{};
    return (int64_t)v;
}

// usize::from_str of the decoded DUP count
uint64_t parse_usize(const std::string& s) {
    size_t i = 0;
    if (i < s.size() && s[i] == '+') ++i;
    if (i == s.size()) throw Fail{};
    unsigned __int128 v = 0;
    for (; i < s.size(); ++i) {
        if (!is_digit(s[i])) throw Fail{};
        v = v * 10 + (unsigned)(s[i] - '0');
        if (v > UINT64_MAX) throw Fail{};
    }
    return (uint64_t)v;
}

// DIF / DUP leading characters (jcampdx.rs:990-1049)
std::string dif_digits(const char* p, size_t n) {
    static const char* pos = "%JKLMNOPQR";
    std::string d;
    const char c = p[0];
    if (c >= 'j' && c <= 'r') d = "-" + std::to_string(c - 'j' + 1);
    else d = std::to_string((int)(std::strchr(pos, c) - pos));
    d.append(p + 1, n - 1);
    return d;
}
std::string dup_digits(const char* p, size_t n) {
    std::string d = std::to_string(p[0] == 's' ? 9 : p[0] - 'S' + 1);
    d.append(p + 1, n - 1);
    return d;
}
// jcampdx.rs:1055-1091: the count minus one, re-encoded ("" for 0)
std::string decrement_dup(const char* p, size_t n) {
    const uint64_t v = parse_usize(dup_digits(p, n));
    if (v == 0) throw Fail{};  // usize underflow: the reference panics
    const std::string dec = std::to_string(v - 1);
    static const char* enc = "STUVWXYZs";
    std::string out;
    if (dec[0] != '0') out.push_back(enc[dec[0] - '1']);
    out.append(dec, 1, std::string::npos);
    return out;
}

template <class C>
inline size_t run(const std::string& s, size_t i, C cls) {
    const size_t n = s.size();
    const char* d = s.data();
    while (i < n && cls(d[i])) ++i;
    return i;
}
struct WsC {
    bool operator()(char c) const { return is_ws(c); }
};
struct DigitC {
    bool operator()(char c) const { return is_digit(c); }
};
struct SignC {
    bool operator()(char c) const { return c == '+' || c == '-'; }
};
struct DifC {
    bool operator()(char c) const { return is_dif(c); }
};
struct DupC {
    bool operator()(char c) const { return is_dup(c); }
};
constexpr WsC ws_c{};
constexpr DigitC digit_c{};
constexpr SignC sign_c{};

// re[0] " $asdf", re[1] " $pac", re[2] the SQZ digits (jcampdx.rs:926-930)
std::string passes_012(const std::string& in) {
    std::string a;
    a.reserve(in.size() * 2);
    for (char c : in) {
        if (is_asdf(c)) a.push_back(' ');
        a.push_back(c);
    }
    std::string b;
    b.reserve(a.size() + a.size() / 4);
    for (size_t i = 0; i < a.size();) {
        if ((a[i] == '+' || a[i] == '-') && i + 1 < a.size() && is_digit(a[i + 1])) {
            b.push_back(' ');
            b.push_back(a[i]);
            b.push_back(a[i + 1]);
            i += 2;
        } else {
            b.push_back(a[i++]);
        }
    }
    std::string c;
    c.reserve(b.size() + b.size() / 4);
    for (char ch : b) {
        if (!is_sqz(ch)) c.push_back(ch);
        else if (ch == '@') c.push_back('0');
        else if (ch >= 'A' && ch <= 'I') c.push_back((char)('1' + (ch - 'A')));
        else {
            c.push_back('-');
            c.push_back((char)('1' + (ch - 'a')));
        }
    }
    return c;
}

// re[3]: \s+(?P<dif>[%J-Rj-r]\d*)\s*(?P<dup>([S-Zs]\d*)?)\s*((\r\n|\n|\r)\s*(?P<next>\d+))
// At a whitespace run W starting at p the backtracking engine's first success is:
// W maximal, the DIF token with all its digits, then the maximal whitespace run R,
// ending at e; if s[e] is a DUP character: the DUP token with all its digits, then a
// maximal whitespace run T that must hold a line break and end at a digit; else R
// must hold a line break and s[e] must be a digit. (Shorter runs or digit counts
// leave a character the next item cannot take.) `next` is then the digit run.
void pass_3(const std::string& s, std::string& out) {
    out.clear();
    size_t i = 0, copied = 0;
    auto has_nl = [&](size_t a, size_t b) {
        for (size_t k = a; k < b; ++k)
            if (s[k] == '\n' || s[k] == '\r') return true;
        return false;
    };
    while (i < s.size()) {
        if (!is_ws(s[i])) {
            ++i;
            continue;
        }
        const size_t p = i, w1 = run(s, p, ws_c);
        bool ok = false;
        size_t dif0 = 0, dif1 = 0, dup0 = 0, dup1 = 0, nx0 = 0, nx1 = 0;
        if (w1 < s.size() && is_dif(s[w1])) {
            dif0 = w1;
            dif1 = run(s, w1 + 1, digit_c);
            const size_t e = run(s, dif1, ws_c);
            if (e < s.size() && is_dup(s[e])) {
                dup0 = e;
                dup1 = run(s, e + 1, digit_c);
                const size_t t = run(s, dup1, ws_c);
                if (t < s.size() && is_digit(s[t]) && has_nl(dup1, t)) {
                    ok = true;
                    nx0 = t;
                }
            } else if (e < s.size() && is_digit(s[e]) && has_nl(dif1, e)) {
                ok = true;
                dup0 = dup1 = e;
                nx0 = e;
            }
        }
        if (!ok) {
            i = w1;  // no match starts inside this whitespace run (the same continuation)
            continue;
        }
        nx1 = run(s, nx0, digit_c);
        out.append(s, copied, p - copied);
        const std::string nxt = s.substr(nx0, nx1 - nx0);
        const size_t dl = dup1 - dup0;
        if (dl == 0 || (dl == 1 && s[dup0] == 'S')) {
            out += " \n" + nxt;
        } else {
            out += " " + s.substr(dif0, dif1 - dif0) + " " + decrement_dup(s.data() + dup0, dl) + " \n" + nxt;
        }
        i = copied = nx1;
    }
    out.append(s, copied, std::string::npos);
}

// The first match of \s+(?P<val>[+-]*\d*|\d+ with sign)\s+(?P<tok>CLS\d*) at or after a
// whitespace run start, as a backtracking engine finds it: items 1-4 are
// [\s]{1,} [+-]{0,} [\d]{MIN,} [\s]{1,} then the token's class character. Returns
// false when no match starts in the run at p.
struct M4 {
    size_t start, val0, val1, tok0, tok1;
};
// Linear in the run: the token class never holds whitespace, so after a \s+ that
// ends at a whitespace-run end only the run's next character can start the token
// (no loop over shorter second runs), and a first \s+ shorter than its run leaves an
// empty value followed by the rest of the same run (one check for all of them, ADVICE
// r4: the nested loops were quadratic in a long whitespace run).
template <class TokC>
bool match_at(const std::string& s, size_t p, int dmin, TokC tokc, M4& m) {
    const size_t wmax = run(s, p, ws_c);
    auto token_after = [&](size_t d, size_t& w2) {  // \s+ then the token's first character
        w2 = run(s, d, ws_c);
        return w2 > d && w2 < s.size() && tokc(s[w2]);
    };
    size_t w2;
    {  // \s+ greedy: the whole run first
        const size_t w = wmax;
        const size_t smax = run(s, w, sign_c);
        for (size_t sg = smax + 1; sg-- > w;) {  // [+-]* greedy
            const size_t dmax = run(s, sg, digit_c);
            for (size_t d = dmax + 1; d-- > sg;) {  // \d* (or \d+) greedy
                if ((int)(d - sg) < dmin) break;
                if (token_after(d, w2)) {
                    m.start = p;
                    m.val0 = w;
                    m.val1 = d;
                    m.tok0 = w2;
                    m.tok1 = run(s, w2 + 1, digit_c);
                    return true;
                }
                // the signs and digits shorter: the next item starts on a sign or digit
            }
        }
    }
    // \s+ shorter than the run (w in (p, wmax)): s[w] is whitespace, so the sign and
    // digit items are empty (no match when digits are required), and the second \s+
    // is the rest of the run -- the same candidate for every such w; greedy takes the
    // longest first \s+, w = wmax - 1
    if (dmin == 0 && wmax >= p + 2 && token_after(wmax - 1, w2)) {
        m.start = p;
        m.val0 = m.val1 = wmax - 1;
        m.tok0 = w2;
        m.tok1 = run(s, w2 + 1, digit_c);
        return true;
    }
    return false;
}
// re[4] (dif) or re[5] (dup) over the whole text; *matched tells whether any matched
void pass_45(const std::string& s, bool dif, bool* matched, std::string& out) {
    out.clear();
    size_t i = 0, copied = 0;
    *matched = false;
    while (i < s.size()) {
        if (!is_ws(s[i])) {
            ++i;
            continue;
        }
        M4 m;
        if (!(dif ? match_at(s, i, 0, DifC{}, m) : match_at(s, i, 1, DupC{}, m))) {
            i = run(s, i, ws_c);
            continue;
        }
        *matched = true;
        out.append(s, copied, m.start - copied);
        if (dif) {  // jcampdx.rs:1020-1049: " value value+difference"
            const int64_t v = parse_i64(s.substr(m.val0, m.val1 - m.val0));
            const int64_t d = parse_i64(dif_digits(s.data() + m.tok0, m.tok1 - m.tok0));
            int64_t r;
            if (__builtin_add_overflow(v, d, &r)) throw Fail{};  // the reference panics
            char buf[48];
            const int k = std::snprintf(buf, sizeof buf, " %lld %lld", (long long)v, (long long)r);
            out.append(buf, (size_t)k);
        } else {  // jcampdx.rs:990-1014: " value" repeated
            const uint64_t k = parse_usize(dup_digits(s.data() + m.tok0, m.tok1 - m.tok0));
            if (k > (uint64_t)1 << 28) throw Fail{};
            for (uint64_t r = 0; r < k; ++r) {
                out.push_back(' ');
                out.append(s, m.val0, m.val1 - m.val0);
            }
        }
        i = copied = m.tok1;
    }
    out.append(s, copied, std::string::npos);
}

bool any_match(const std::string& s, bool dif) {
    M4 m;
    for (size_t i = 0; i < s.size();) {
        if (!is_ws(s[i])) {
            ++i;
            continue;
        }
        if (dif ? match_at(s, i, 0, DifC{}, m) : match_at(s, i, 1, DupC{}, m)) return true;
        i = run(s, i, ws_c);
    }
    return false;
}

// f64::from_str: [+-]?(digits[.digits]|.digits)([eE][+-]?digits)? or inf/infinity/nan
double parse_f64(const char* p, size_t n) {
    size_t i = 0;
    if (i < n && (p[i] == '+' || p[i] == '-')) ++i;
    auto word = [&](const char* w) {
        const size_t L = std::strlen(w);
        if (n - i != L) return false;
        for (size_t k = 0; k < L; ++k)
            if ((p[i + k] | 0x20) != w[k]) return false;
        return true;
    };
    const bool neg = n > 0 && p[0] == '-';
    if (word("inf") || word("infinity")) return neg ? -INFINITY : INFINITY;
    if (word("nan")) throw Fail{};  // NaN payload/sign: left to the Python reader
    const size_t d0 = i;
    while (i < n && is_digit(p[i])) ++i;
    const size_t id = i - d0;
    size_t fd = 0;
    if (i < n && p[i] == '.') {
        ++i;
        const size_t f0 = i;
        while (i < n && is_digit(p[i])) ++i;
        fd = i - f0;
    }
    if (id == 0 && fd == 0) throw Fail{};
    if (i < n && (p[i] == 'e' || p[i] == 'E')) {
        ++i;
        if (i < n && (p[i] == '+' || p[i] == '-')) ++i;
        const size_t e0 = i;
        while (i < n && is_digit(p[i])) ++i;
        if (i == e0) throw Fail{};
    }
    if (i != n) throw Fail{};
    // correctly rounded, like Rust's parse (glibc strtod rounds correctly)
    const std::string tok(p, n);
    errno = 0;
    return std::strtod(tok.c_str(), nullptr);  // ERANGE: +-inf or a (correctly rounded) subnormal/0
}

// jcampdx.rs:892-916: str::lines, split_whitespace, skip(1), parse, * factor
void decode_affn(const std::string& s, double factor, std::vector<double>& out) {
    size_t ls = 0;
    while (ls < s.size()) {
        size_t le = s.find('\n', ls);
        const size_t next = le == std::string::npos ? s.size() : le + 1;
        if (le == std::string::npos) le = s.size();
        size_t end = le;
        if (end > ls && s[end - 1] == '\r') --end;  // lines() strips one trailing \r
        bool first = true;
        for (size_t i = ls; i < end;) {
            while (i < end && is_ws(s[i])) ++i;
            if (i >= end) break;
            size_t j = i;
            while (j < end && !is_ws(s[j])) ++j;
            if (!first) out.push_back(parse_f64(s.data() + i, j - i) * factor);
            first = false;
            i = j;
        }
        ls = next;
    }
}

}  // namespace

extern "C" int mdg_jcampdx_decode(const char* data, size_t len, double factor, double* out, size_t cap,
                                  size_t* n_out) {
    if ((!data && len) || !n_out || (!out && cap)) return MDG_INVALID_ARGUMENT;
    *n_out = 0;
    for (size_t k = 0; k < len; ++k)
        if ((unsigned char)data[k] >= 0x80) return MDG_INVALID_ARGUMENT;  // Unicode classes
    std::vector<double> v;
    try {
        std::string s(data, len);
        bool asdf = false;
        for (char c : s) asdf = asdf || is_asdf(c);
        if (asdf) {  // jcampdx.rs:925-966
            std::string t;  // ping-pong buffers: the passes reuse their capacity
            s = passes_012(s);
            t.reserve(2 * s.size());
            pass_3(s, t);
            s.swap(t);
            s.reserve(2 * t.capacity());
            for (;;) {
                bool m4 = false, m5 = false;
                pass_45(s, true, &m4, t);
                pass_45(t, false, &m5, s);
                if (!any_match(s, true) && !any_match(s, false)) break;
            }
        }
        decode_affn(s, factor, v);
    } catch (const Fail&) {
        return MDG_INVALID_ARGUMENT;
    } catch (...) {
        return MDG_ERR_OUT_OF_MEMORY;
    }
    *n_out = v.size();
    if (v.size() > cap) return MDG_CAPACITY;
    if (!v.empty()) std::memcpy(out, v.data(), v.size() * sizeof(double));
    return MDG_OK;
}
