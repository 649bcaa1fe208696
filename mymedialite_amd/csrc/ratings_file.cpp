// ratings_file.cpp -- parallel reader for MyMediaLite rating files (host code of libmml_hip.so).
//
// Restates IO/StaticRatingData.Read (src/MyMediaLite/IO/StaticRatingData.cs:36-117) for files
// far larger than the reference's single-threaded StreamReader handles well (at C4
// the text parse of 1 B lines dominates wall time):
//   * lines as TextReader.ReadLine splits them ("\n" or "\r\n"); the first line skipped with
//     ignore_first_line; empty lines skipped; size = the line count (arrays sized by it);
//   * tokens split on every '\t', ' ' and ',' (Constants.SPLIT_CHARS: consecutive separators give
//     empty tokens, exactly like String.Split); >= 3 tokens or a FormatException;
//   * ids: IdentityMapping (int.Parse) or Mapping.ToInternalID (Data/Mapping.cs:75-85: a new
//     external id gets the next internal id, in first-appearance order), optionally seeded with
//     the ids a mapping already holds; ratings: float.Parse (InvariantCulture), correctly rounded.
// ReadLine ends a line at "\n", "\r" or "\r\n"; ItemData.Read (IO/ItemData.cs:59-94) is the
// same parse with two columns and Trim()-blank lines skipped (MML_READ_ITEM_DATA).
// The file is read once; T threads own contiguous byte chunks: pass 1 counts lines, pass 2
// tokenises into the final arrays; Mapping columns are resolved by hash partition (map_column), with
// ids assigned in first-appearance order, so the internal ids equal the sequential reader's.
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "mml_internal.h"


namespace {

struct Key {  // an id token in the file buffer (or a seed string)
    const char* p;
    uint32_t n;
};

inline bool is_sep(char c) { return c == '\t' || c == ' ' || c == ','; }

// String.Split(SPLIT_CHARS) restricted to the first `want` tokens; false if there are fewer.
inline bool split_first(std::string_view s, std::string_view (&tok)[3], int want) {
    size_t start = 0;
    int n = 0;
    for (size_t x = 0; x <= s.size() && n < want; ++x) {
        if (x == s.size() || is_sep(s[x])) {
            tok[n++] = s.substr(start, x - start);
            start = x + 1;
        }
    }
    return n == want;
}

// line.Trim().Length == 0: every character is Char.IsWhiteSpace (U+0009-000D, U+0020, U+0085,
// U+00A0, U+1680, U+2000-200A, U+2028, U+2029, U+202F, U+205F, U+3000), decoded from UTF-8
inline bool is_blank(std::string_view s) {
    const auto* b = (const unsigned char*)s.data();
    const size_t n = s.size();
    for (size_t x = 0; x < n;) {
        const unsigned c = b[x];
        if (c == ' ' || (c >= 0x09 && c <= 0x0D)) {
            ++x;
        } else if (c == 0xC2 && x + 1 < n && (b[x + 1] == 0x85 || b[x + 1] == 0xA0)) {
            x += 2;
        } else if (c == 0xE1 && x + 2 < n && b[x + 1] == 0x9A && b[x + 2] == 0x80) {
            x += 3;
        } else if (c == 0xE2 && x + 2 < n && b[x + 1] == 0x80 &&
                   (b[x + 2] <= 0x8A || b[x + 2] == 0xA8 || b[x + 2] == 0xA9 || b[x + 2] == 0xAF) &&
                   b[x + 2] >= 0x80) {
            x += 3;
        } else if (c == 0xE2 && x + 2 < n && b[x + 1] == 0x81 && b[x + 2] == 0x9F) {
            x += 3;
        } else if (c == 0xE3 && x + 2 < n && b[x + 1] == 0x80 && b[x + 2] == 0x80) {
            x += 3;
        } else {
            return false;
        }
    }
    return true;
}

inline bool parse_int(std::string_view t, int32_t& out) {  // int.Parse (invariant): [+-]digits
    if (!t.empty() && t[0] == '+') t.remove_prefix(1);
    const auto r = std::from_chars(t.data(), t.data() + t.size(), out);
    return r.ec == std::errc() && r.ptr == t.data() + t.size();
}

inline bool parse_float(std::string_view t, float& out) {  // float.Parse (InvariantCulture)
    if (!t.empty() && t[0] == '+') t.remove_prefix(1);
    const auto r = std::from_chars(t.data(), t.data() + t.size(), out);
    return r.ec == std::errc() && r.ptr == t.data() + t.size();
}

inline uint64_t hash_bytes(const char* p, size_t n) {  // FNV-1a 64, then a murmur finaliser
    uint64_t h = 1469598103934665603ull;
    for (size_t x = 0; x < n; ++x) h = (h ^ (uint8_t)p[x]) * 1099511628211ull;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    return h;
}

// which of T partitions owns a key: the high hash bits (the table index uses the low ones)
inline int part_of(uint64_t h, int T) { return (int)(((h >> 32) * (uint64_t)T) >> 32); }

// One partition of an id column: an open-addressing table (linear probing, power-of-two
// capacity, at most half full) from key to a dense key number; per key number the key, the line
// it first appears on (-1 for a seed) and, after the merge, its internal id.
struct Partition {
    struct Slot {
        uint64_t h;
        const char* p;
        uint32_t n;
        int32_t num;  // -1: empty
    };
    std::vector<Slot> slots = std::vector<Slot>(1024, Slot{0, nullptr, 0, -1});
    std::vector<Key> keys;
    std::vector<int64_t> first;
    std::vector<int32_t> id;
    // the key number of (p, n), inserted with first appearance `line` if absent
    int32_t lookup_insert(const char* p, uint32_t n, uint64_t h, int64_t line) {
        if (2 * (keys.size() + 1) > slots.size()) grow();
        const size_t m = slots.size() - 1;
        for (size_t x = h & m;; x = (x + 1) & m) {
            Slot& s = slots[x];
            if (s.num < 0) {
                s = Slot{h, p, n, (int32_t)keys.size()};
                keys.push_back(Key{p, n});
                first.push_back(line);
                return s.num;
            }
            if (s.h == h && s.n == n && std::memcmp(s.p, p, n) == 0) return s.num;
        }
    }
    void grow() {
        std::vector<Slot> old(slots.size() * 2, Slot{0, nullptr, 0, -1});
        old.swap(slots);
        const size_t m = slots.size() - 1;
        for (const Slot& s : old)
            if (s.num >= 0) {
                size_t x = s.h & m;
                while (slots[x].num >= 0) x = (x + 1) & m;
                slots[x] = s;
            }
    }
};

// Mapping.ToInternalID over a whole column: seeds keep ids 0..n_seed-1, new keys get n_seed,
// n_seed + 1, ... in order of first appearance.  T threads each own one hash partition and scan
// the column's hashes in file order (so a partition's new keys are ordered by first line); the
// partitions' new-key lists are then merged by first line, and every line's id resolved.
void map_column(const uint64_t* hash, const Key* key, int64_t N, const char* const* seed,
                int32_t n_seed, int T, const std::vector<int64_t>& at, int32_t* out,
                std::vector<std::string>& fresh) {
    std::vector<Partition> part(T);
    std::unique_ptr<int32_t[]> num(new int32_t[N]);
    std::vector<std::thread> th;
    for (int p = 0; p < T; ++p)
        th.emplace_back([&, p] {
            Partition& P = part[p];
            for (int32_t x = 0; x < n_seed; ++x) {
                const uint32_t n = (uint32_t)std::strlen(seed[x]);
                const uint64_t h = hash_bytes(seed[x], n);
                if (part_of(h, T) == p) {
                    P.lookup_insert(seed[x], n, h, -1);
                    P.id.push_back(x);
                }
            }
            for (int64_t o = 0; o < N; ++o)
                if (part_of(hash[o], T) == p)
                    num[o] = P.lookup_insert(key[o].p, key[o].n, hash[o], o);
            P.id.resize(P.keys.size(), -1);
        });
    for (auto& t : th) t.join();
    th.clear();
    // merge the partitions' new keys by first appearance
    std::vector<size_t> head(T);
    for (int p = 0; p < T; ++p) {
        head[p] = 0;
        while (head[p] < part[p].first.size() && part[p].first[head[p]] < 0) ++head[p];
    }
    int32_t next = n_seed;
    for (;;) {
        int best = -1;
        int64_t bf = 0;
        for (int p = 0; p < T; ++p)
            if (head[p] < part[p].first.size() && (best < 0 || part[p].first[head[p]] < bf)) {
                best = p;
                bf = part[p].first[head[p]];
            }
        if (best < 0) break;
        Partition& P = part[best];
        P.id[head[best]] = next++;
        fresh.emplace_back(P.keys[head[best]].p, P.keys[head[best]].n);
        ++head[best];
    }
    for (int c = 0; c < T; ++c)
        th.emplace_back([&, c] {
            for (int64_t o = at[c]; o < at[c + 1]; ++o) out[o] = part[part_of(hash[o], T)].id[num[o]];
        });
    for (auto& t : th) t.join();
}

}  // namespace

using mml::guard;

namespace {

// FileSerializer's cache restated for the native reader: header "MMLRAT01", the flags that shape
// the parse, n_lines, n_ratings, then users[], items[], values[] (host byte order).
constexpr char kCacheMagic[8] = {'M', 'M', 'L', 'R', 'A', 'T', '0', '1'};
constexpr int32_t kCacheFlagMask = MML_READ_IGNORE_FIRST_LINE | MML_READ_WITHOUT_RATINGS |
                                   MML_READ_ITEM_DATA;

// [0, bytes) split over T threads, fn(lo, hi) each (the page faults of fresh arrays and the
// copies then run in parallel: a single thread moves ~2-3 GB/s)
template <class F>
void parallel_ranges(size_t bytes, int T, F&& fn) {
    T = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, T), bytes >> 24));
    if (T == 1) return (void)fn((size_t)0, bytes);
    std::vector<std::thread> th;
    for (int c = 0; c < T; ++c)
        th.emplace_back([&, c] { fn(bytes * c / T & ~(size_t)4095, c + 1 == T ? bytes
                                                                          : bytes * (c + 1) / T & ~(size_t)4095); });
    for (auto& t : th) t.join();
}

void parallel_copy(void* dst, const void* src, size_t bytes, int T) {
    parallel_ranges(bytes, T, [&](size_t lo, size_t hi) {
        std::memcpy(static_cast<char*>(dst) + lo, static_cast<const char*>(src) + lo, hi - lo);
    });
}

// [off, off + bytes) of fd into dst with pread on T threads; false on a short read
bool parallel_pread(int fd, void* dst, size_t bytes, off_t off, int T) {
    std::atomic<bool> ok{true};
    parallel_ranges(bytes, T, [&](size_t lo, size_t hi) {
        while (lo < hi && ok) {
            const ssize_t r = pread(fd, static_cast<char*>(dst) + lo,
                                    std::min<size_t>(hi - lo, (size_t)1 << 30), off + (off_t)lo);
            if (r <= 0) ok = false;
            else lo += (size_t)r;
        }
    });
    return ok;
}

bool load_cache(const std::string& bin, int32_t flags, mml_rating_file& f) {
    const int fd = open(bin.c_str(), O_RDONLY);
    if (fd < 0) return false;
    struct Closer {
        int fd;
        ~Closer() { close(fd); }
    } closer{fd};
    char head[8 + 4 + 8 + 8];
    if (pread(fd, head, sizeof head, 0) != (ssize_t)sizeof head) return false;
    int32_t fl = 0;
    int64_t nl = 0, nr = 0;
    std::memcpy(&fl, head + 8, sizeof fl);
    std::memcpy(&nl, head + 12, sizeof nl);
    std::memcpy(&nr, head + 20, sizeof nr);
    if (std::memcmp(head, kCacheMagic, 8) != 0 || fl != (flags & kCacheFlagMask) || nr < 0 ||
        nl < nr)
        return false;
    f.n_lines = nl;
    f.n_ratings = nr;
    f.users.reset(new int32_t[std::max<int64_t>(1, nr)]);
    f.items.reset(new int32_t[std::max<int64_t>(1, nr)]);
    f.values.reset(new float[std::max<int64_t>(1, nr)]);
    const size_t b = sizeof(int32_t) * (size_t)nr;
    const off_t o = (off_t)sizeof head;
    return parallel_pread(fd, f.users.get(), b, o, f.threads) &&
           parallel_pread(fd, f.items.get(), b, o + (off_t)b, f.threads) &&
           parallel_pread(fd, f.values.get(), b, o + 2 * (off_t)b, f.threads);
}

void save_cache(const std::string& bin, int32_t flags, const mml_rating_file& f) {
    // FileSerializer.CanWrite: no writable location, no cache
    const std::string tmp = bin + ".tmp";
    {
        std::ofstream out(tmp, std::ios::binary | std::ios::trunc);
        if (!out) return;
        const int32_t fl = flags & kCacheFlagMask;
        out.write(kCacheMagic, 8);
        out.write(reinterpret_cast<const char*>(&fl), sizeof fl);
        out.write(reinterpret_cast<const char*>(&f.n_lines), sizeof f.n_lines);
        out.write(reinterpret_cast<const char*>(&f.n_ratings), sizeof f.n_ratings);
        out.write(reinterpret_cast<const char*>(f.users.get()),
                  (std::streamsize)(sizeof(int32_t) * f.n_ratings));
        out.write(reinterpret_cast<const char*>(f.items.get()),
                  (std::streamsize)(sizeof(int32_t) * f.n_ratings));
        out.write(reinterpret_cast<const char*>(f.values.get()),
                  (std::streamsize)(sizeof(float) * f.n_ratings));
        if (!out) {
            std::remove(tmp.c_str());
            return;
        }
    }
    std::rename(tmp.c_str(), bin.c_str());  // readers never see a partial cache
}

}  // namespace

extern "C" mml_status mml_rating_file_read(const char* path, int32_t flags, int32_t n_threads,
                                           const char* const* user_seed, int32_t n_user_seed,
                                           const char* const* item_seed, int32_t n_item_seed,
                                           mml_rating_file** out) {
    return guard([&] {
        MML_REQUIRE(path && out, "null argument");
        MML_REQUIRE(n_user_seed >= 0 && n_item_seed >= 0, "bad seed counts");
        const bool skip_first = flags & MML_READ_IGNORE_FIRST_LINE;
        const bool user_identity = flags & MML_READ_USER_IDENTITY;
        const bool item_identity = flags & MML_READ_ITEM_IDENTITY;
        const bool item_data = flags & MML_READ_ITEM_DATA;
        const int want = item_data || (flags & MML_READ_WITHOUT_RATINGS) ? 2 : 3;
        std::unique_ptr<mml_rating_file> f(new mml_rating_file());
        f->threads = std::max(1, std::min<int>(n_threads > 0 ? n_threads : 8, 64));
        // FileSerializer.Should: neither column uses a Mapping
        const bool use_cache = (flags & MML_READ_BINARY_CACHE) && user_identity && item_identity;
        const std::string bin =
            std::string(path) + (item_data ? ".bin.mml.PosOnlyFeedback" : ".bin.mml.StaticRatings");
        if (use_cache && load_cache(bin, flags, *f)) {
            *out = f.release();
            return;
        }
        size_t n = 0;
        std::unique_ptr<char[]> text;
        {
            std::ifstream in(path, std::ios::binary);
            if (!in) mml::fail(MML_ERR_ARG, std::string("cannot open ") + path);
            in.seekg(0, std::ios::end);
            n = (size_t)in.tellg();
            in.seekg(0);
            text.reset(new char[n + 1]);
            if (n > 0) in.read(text.get(), (std::streamsize)n);
        }
        const char* base = text.get();
        // StreamReader drops a UTF-8 byte-order mark
        const size_t bom = n >= 3 && std::memcmp(base, "\xEF\xBB\xBF", 3) == 0 ? 3 : 0;
        const int T = std::max(1, std::min<int>(n_threads > 0 ? n_threads : 8, 64));
        // Thread c owns the lines that START in its byte range [n c / T, n (c + 1) / T): a line
        // starts at the BOM's end or after "\n", a lone "\r" or "\r\n" (ReadLine strips them; a
        // last unterminated line counts); fn(line) sees them in order, the skipped first excepted.
        auto is_start = [&](size_t p) {
            return p == bom ||
                   (p > bom && (base[p - 1] == '\n' || (base[p - 1] == '\r' && base[p] != '\n')));
        };
        auto for_each_line = [&](int c, auto&& fn) {
            const size_t hi = n * (c + 1) / T;
            size_t s = n * c / T;
            while (s < hi && !is_start(s)) ++s;
            while (s < hi && s < n) {
                const void* nlp = std::memchr(base + s, '\n', n - s);
                size_t e = nlp ? (size_t)((const char*)nlp - base) : n;  // line end
                size_t next = e + 1;                                        // next line start
                if (const void* crp = std::memchr(base + s, '\r', e - s)) {
                    const size_t r = (size_t)((const char*)crp - base);
                    next = r + 1 == e ? e + 1 : r + 1;  // "\r\n" or a lone "\r"
                    e = r;
                }
                const bool skip = skip_first && s == bom;
                const size_t s0 = s;
                s = next;
                if (!skip && !fn(std::string_view(base + s0, e - s0))) return;
            }
        };
        auto is_empty = [&](std::string_view line) {
            return item_data ? is_blank(line) : line.empty();
        };
        std::vector<std::thread> th;
        auto parallel = [&](auto&& body) {
            for (int c = 0; c < T; ++c) th.emplace_back([&, c] { body(c); });
            for (auto& t : th) t.join();
            th.clear();
        };
        // ---- pass 1: lines and non-empty lines per chunk -> each chunk's output offset
        std::vector<int64_t> lines(T, 0), at(T + 1, 0);
        parallel([&](int c) {
            int64_t nl = 0, nr = 0;
            for_each_line(c, [&](std::string_view line) {
                ++nl;
                nr += !is_empty(line);
                return true;
            });
            lines[c] = nl;
            at[c + 1] = nr;
        });
        for (int c = 0; c < T; ++c) {
            f->n_lines += lines[c];
            at[c + 1] += at[c];
        }
        const int64_t N = at[T];
        f->n_ratings = N;
        f->users.reset(new int32_t[N]);
        f->items.reset(new int32_t[N]);
        f->values.reset(new float[N]);
        std::unique_ptr<uint64_t[]> uh, ih;
        std::unique_ptr<Key[]> uk, ik;
        if (!user_identity) uh.reset(new uint64_t[N]), uk.reset(new Key[N]);
        if (!item_identity) ih.reset(new uint64_t[N]), ik.reset(new Key[N]);
        // ---- pass 2: tokenise into the output arrays (identity ids and ratings parsed here;
        //      Mapping ids kept as key + hash); the first error of the first failing chunk is
        //      the first error in the file, as the sequential reader throws it
        std::vector<std::string> err(T);
        parallel([&](int c) {
            int64_t o = at[c];
            for_each_line(c, [&](std::string_view line) {
                if (is_empty(line)) return true;
                std::string_view tok[3];
                if (!split_first(line, tok, want)) {
                    err[c] = "Expected at least " + std::to_string(want) +
                             " columns: " + std::string(line);
                    return false;
                }
                // ItemData wraps every parse failure as "Could not read line '...'"
                auto bad = [&](const char* what, std::string_view t) {
                    err[c] = item_data ? "Could not read line '" + std::string(line) + "'"
                                       : std::string("cannot parse ") + what + " '" +
                                             std::string(t) + "'";
                    return false;
                };
                if (user_identity) {
                    if (!parse_int(tok[0], f->users[o])) return bad("user id", tok[0]);
                } else {
                    uk[o] = Key{tok[0].data(), (uint32_t)tok[0].size()};
                    uh[o] = hash_bytes(tok[0].data(), tok[0].size());
                }
                if (item_identity) {
                    if (!parse_int(tok[1], f->items[o])) return bad("item id", tok[1]);
                } else {
                    ik[o] = Key{tok[1].data(), (uint32_t)tok[1].size()};
                    ih[o] = hash_bytes(tok[1].data(), tok[1].size());
                }
                if (want == 3) {
                    if (!parse_float(tok[2], f->values[o])) return bad("rating", tok[2]);
                } else {
                    f->values[o] = 0.0f;
                }
                ++o;
                return true;
            });
        });
        for (int c = 0; c < T; ++c) MML_REQUIRE(err[c].empty(), err[c]);
        // ---- Mapping columns
        if (!user_identity)
            map_column(uh.get(), uk.get(), N, user_seed, n_user_seed, T, at, f->users.get(),
                       f->new_users);
        if (!item_identity)
            map_column(ih.get(), ik.get(), N, item_seed, n_item_seed, T, at, f->items.get(),
                       f->new_items);
        if (use_cache) save_cache(bin, flags, *f);
        *out = f.release();
    });
}

extern "C" mml_status mml_rating_file_counts(mml_rating_file* f, int64_t* n_ratings,
                                             int64_t* n_lines, int32_t* n_new_users,
                                             int32_t* n_new_items) {
    return guard([&] {
        MML_REQUIRE(f && n_ratings && n_lines && n_new_users && n_new_items, "null argument");
        *n_ratings = f->n_ratings;
        *n_lines = f->n_lines;
        *n_new_users = (int32_t)f->new_users.size();
        *n_new_items = (int32_t)f->new_items.size();
    });
}

extern "C" mml_status mml_rating_file_get(mml_rating_file* f, int32_t* users, int32_t* items,
                                          float* values) {
    return guard([&] {
        MML_REQUIRE(f && users && items && values, "null argument");
        if (!f->users && f->ctx) {  // parsed on the device: the arrays live in HBM
            f->ctx->activate();
            const size_t n = (size_t)f->n_ratings;
            if (n > 0) {
                MML_HIP(hipMemcpy(users, f->d_users.get(), sizeof(int32_t) * n,
                                  hipMemcpyDeviceToHost));
                MML_HIP(hipMemcpy(items, f->d_items.get(), sizeof(int32_t) * n,
                                  hipMemcpyDeviceToHost));
                MML_HIP(hipMemcpy(values, f->d_values.get(), sizeof(float) * n,
                                  hipMemcpyDeviceToHost));
            }
            return;
        }
        parallel_copy(users, f->users.get(), sizeof(int32_t) * f->n_ratings, f->threads);
        parallel_copy(items, f->items.get(), sizeof(int32_t) * f->n_ratings, f->threads);
        parallel_copy(values, f->values.get(), sizeof(float) * f->n_ratings, f->threads);
    });
}

// All new external ids of one column (which = 0 users, 1 items) in internal-id order, each followed
// by '\n' (ids never contain one: the file is split into lines first); *bytes = the total length
// (call with cap = 0 to query).
extern "C" mml_status mml_rating_file_new_ids(mml_rating_file* f, int32_t which, char* buf,
                                              int64_t cap, int64_t* bytes) {
    return guard([&] {
        MML_REQUIRE(f && bytes && (which == 0 || which == 1), "bad argument");
        const auto& v = which == 0 ? f->new_users : f->new_items;
        int64_t n = 0;
        for (const auto& x : v) n += (int64_t)x.size() + 1;
        *bytes = n;
        if (cap > 0) {
            MML_REQUIRE(buf && cap >= n, "buffer too small");
            char* o = buf;
            for (const auto& x : v) {
                std::memcpy(o, x.data(), x.size());
                o += x.size();
                *o++ = '\n';
            }
        }
    });
}

extern "C" mml_status mml_rating_file_destroy(mml_rating_file* f) {
    return guard([&] {
        if (f && f->ctx) (void)hipSetDevice(f->ctx->device);  // its HBM arrays are freed here
        delete f;
    });
}
