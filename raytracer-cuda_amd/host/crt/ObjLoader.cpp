// ObjLoader.cpp — see ObjLoader.h for the semantics restated.
#include "ObjLoader.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <thread>
#include <unordered_map>

#include "ParallelFor.h"

namespace CRT {

static inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
static inline bool is_space(char c) { return c == ' ' || c == '\t'; }

// Number parser following tinyobjloader v1.0's tryParseDouble (the reference's OBJ dependency; tinyobjloader is
// MIT-licensed, Copyright (c) 2012-2016 Syoyo Fujita and many contributors), restated so that vertex coordinates round
// exactly as the reference's loader rounds them.
bool TryParseDouble(const char* s, const char* s_end, double* result) {
    if (s >= s_end) return false;
    double mantissa = 0.0;
    int exponent = 0;
    char sign = '+', exp_sign = '+';
    const char* curr = s;
    int read = 0;
    bool end_not_reached = false;
    if (*curr == '+' || *curr == '-') {
        sign = *curr;
        curr++;
    } else if (is_digit(*curr)) {
    } else {
        return false;
    }
    end_not_reached = (curr != s_end);
    while (end_not_reached && is_digit(*curr)) {
        mantissa *= 10;
        mantissa += static_cast<int>(*curr - 0x30);
        curr++;
        read++;
        end_not_reached = (curr != s_end);
    }
    if (read == 0) return false;
    if (!end_not_reached) goto assemble;
    if (*curr == '.') {
        curr++;
        read = 1;
        end_not_reached = (curr != s_end);
        while (end_not_reached && is_digit(*curr)) {
            static const double pow_lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            const int lut_entries = sizeof pow_lut / sizeof pow_lut[0];
            mantissa += static_cast<int>(*curr - 0x30) * (read < lut_entries ? pow_lut[read] : std::pow(10.0, -read));
            read++;
            curr++;
            end_not_reached = (curr != s_end);
        }
    } else if (*curr == 'e' || *curr == 'E') {
    } else {
        goto assemble;
    }
    if (!end_not_reached) goto assemble;
    if (*curr == 'e' || *curr == 'E') {
        curr++;
        end_not_reached = (curr != s_end);
        if (end_not_reached && (*curr == '+' || *curr == '-')) {
            exp_sign = *curr;
            curr++;
        } else if (end_not_reached && is_digit(*curr)) {
        } else {
            return false;
        }
        read = 0;
        end_not_reached = (curr != s_end);
        while (end_not_reached && is_digit(*curr)) {
            // tinyobjloader lets the int overflow (undefined behaviour, found by UBSan in tools/run_asan.sh); any
            // exponent beyond 9999 already makes the value inf or 0, so it stops growing there
            if (exponent < 100000) exponent = exponent * 10 + static_cast<int>(*curr - 0x30);
            curr++;
            read++;
            end_not_reached = (curr != s_end);
        }
        exponent *= (exp_sign == '+' ? 1 : -1);
        if (read == 0) return false;
    }
assemble:
    *result = (sign == '+' ? 1 : -1) * (exponent ? std::ldexp(mantissa * std::pow(5.0, exponent), exponent) : mantissa);
    return true;
}

namespace {

// tokenizer over one line
struct Tok {
    const char* p;
    const char* end;
    void skip() { while (p < end && is_space(*p)) ++p; }
    bool next(const char** b, const char** e) {
        skip();
        if (p >= end) return false;
        *b = p;
        while (p < end && !is_space(*p)) ++p;
        *e = p;
        return true;
    }
};

float parse_real(Tok& t, double def = 0.0) {
    const char *b, *e;
    double v = def;
    if (t.next(&b, &e)) {
        double r;
        if (TryParseDouble(b, e, &r)) v = r;
    }
    return static_cast<float>(v);
}

bool read_lines(const std::string& path, std::string* buf) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    f.seekg(0, std::ios::end);
    buf->resize((size_t)f.tellg());
    f.seekg(0);
    f.read(&(*buf)[0], (std::streamsize)buf->size());
    return (bool)f || f.eof();
}

template <class F>
void for_each_line(const char* p, const char* end, F&& fn) {
    while (p < end) {
        const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
        const char* le = nl ? nl : end;
        const char* q = le;
        while (q > p && (q[-1] == '\r')) --q;
        fn(p, q);
        p = nl ? nl + 1 : end;
    }
}

bool load_mtl(const std::string& path, std::vector<ObjMaterial>* mats, std::unordered_map<std::string, int>* map) {
    std::string buf;
    if (!read_lines(path, &buf)) return false;
    ObjMaterial cur;
    bool have = false;
    auto push = [&] {
        if (have && !cur.name.empty()) {
            map->insert({cur.name, (int)mats->size()});
            mats->push_back(cur);
        }
    };
    for_each_line(buf.data(), buf.data() + buf.size(), [&](const char* b, const char* e) {
        Tok t{b, e};
        const char *kb, *ke;
        if (!t.next(&kb, &ke) || *kb == '#') return;
        std::string key(kb, ke);
        if (key == "newmtl") {
            push();
            cur = ObjMaterial();
            have = true;
            t.skip();
            cur.name.assign(t.p, t.end);
            while (!cur.name.empty() && is_space(cur.name.back())) cur.name.pop_back();
            return;
        }
        if (!have) return;
        if (key == "Kd") { for (float& c : cur.diffuse) c = parse_real(t); }
        else if (key == "Ks") { for (float& c : cur.specular) c = parse_real(t); }
        else if (key == "Ke") { for (float& c : cur.emission) c = parse_real(t); }
        else if (key == "d") cur.dissolve = parse_real(t);
        else if (key == "Tr") cur.dissolve = 1.0f - parse_real(t);
        else if (key == "Ni") cur.ior = parse_real(t);
        else if (key == "Ns") cur.shininess = parse_real(t);
        else if (key == "Pr") cur.roughness = parse_real(t);
    });
    push();
    return true;
}

// One contiguous run of whole lines of the file, parsed on its own (LoadObj parses a large file in up to 16 of them
// at once).  Everything that depends on the lines before the run is left symbolic and resolved in file order when the
// runs are joined: a negative (relative) face index counts from the run's first vertex, and a face's material is
// "the state after this run's first k usemtl / mtllib lines".
struct Event {
    bool mtllib;
    std::string text;   // usemtl: the material name; mtllib: the rest of the line
};
struct Run {
    std::vector<float> vertices;
    std::vector<int32_t> tri;        // 3 vertex indices per triangle
    std::vector<uint8_t> rel;        // per index: 1 = relative to the run's first vertex (a negative OBJ index)
    std::vector<int32_t> tri_event;  // per triangle: this run's events before its face
    std::vector<Event> events;
    bool zero_index = false;
    void swap_into(Run* o) {   // o takes this (empty) run's storage; o's old storage is freed with *this
        vertices.swap(o->vertices);
        tri.swap(o->tri);
        rel.swap(o->rel);
        tri_event.swap(o->tri_event);
        events.swap(o->events);
    }
};

void parse_run(const char* b, const char* e, Run* R) {
    struct Corner { int32_t v; uint8_t rel; };
    std::vector<Corner> face;
    // capacity for typical lines ("v x y z" >= 8 bytes a vertex, "f a b c" a triangle): fewer reallocations while
    // other threads parse (an unmapped old block interrupts every thread of the process).  Denser files (short
    // integer coordinates, 1-digit indices) still grow the vectors; the capacity is a hint, not a bound
    const size_t bytes = (size_t)(e - b);
    R->vertices.reserve(bytes / 8);
    R->tri.reserve(bytes / 6);
    R->rel.reserve(bytes / 6);
    R->tri_event.reserve(bytes / 18);
    for_each_line(b, e, [&](const char* lb, const char* le) {
        if (R->zero_index) return;
        Tok t{lb, le};
        const char *kb, *ke;
        if (!t.next(&kb, &ke) || *kb == '#') return;
        const size_t kl = (size_t)(ke - kb);
        if (kl == 1 && kb[0] == 'v') {
            R->vertices.push_back(parse_real(t));
            R->vertices.push_back(parse_real(t));
            R->vertices.push_back(parse_real(t));
        } else if (kl == 1 && kb[0] == 'f') {
            const int nv = (int)(R->vertices.size() / 3);
            face.clear();
            const char *fb, *fe;
            while (t.next(&fb, &fe)) {
                int idx = atoi(fb);
                if (idx > 0) face.push_back({idx - 1, 0});
                else if (idx < 0) face.push_back({nv + idx, 1});   // + the vertices before the run, when joined
                else { R->zero_index = true; return; }
            }
            if (face.size() < 3) return;
            Corner i0 = face[0], i1, i2 = face[1];
            for (size_t k = 2; k < face.size(); ++k) {   // fan (0, k-1, k)
                i1 = i2;
                i2 = face[k];
                for (const Corner& c : {i0, i1, i2}) {
                    R->tri.push_back(c.v);
                    R->rel.push_back(c.rel);
                }
                R->tri_event.push_back((int32_t)R->events.size());
            }
        } else if (kl == 6 && memcmp(kb, "usemtl", 6) == 0) {
            t.skip();
            std::string name(t.p, t.end);
            while (!name.empty() && is_space(name.back())) name.pop_back();
            R->events.push_back({false, std::move(name)});
        } else if (kl == 6 && memcmp(kb, "mtllib", 6) == 0) {
            R->events.push_back({true, std::string(t.p, t.end)});
        }
    });
}

// Runs of about `run_bytes` each (CRT_OBJ_RUN_BYTES overrides, for tests), at most 16, cut after a newline.
std::vector<std::pair<const char*, const char*>> split_runs(const std::string& buf) {
    size_t run_bytes = (size_t)4 << 20;
    if (const char* env = std::getenv("CRT_OBJ_RUN_BYTES")) run_bytes = std::max<size_t>(1, std::strtoull(env, nullptr, 10));
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t n = std::max<size_t>(1, std::min<size_t>({(buf.size() + run_bytes - 1) / run_bytes, 16, hw ? hw : 1}));
    std::vector<std::pair<const char*, const char*>> runs;
    const char* p = buf.data();
    const char* end = p + buf.size();
    for (size_t k = 1; k <= n && p < end; ++k) {
        const char* q = k == n ? end : std::max(p, buf.data() + buf.size() * k / n);
        if (q < end) {
            const char* nl = (const char*)memchr(q, '\n', (size_t)(end - q));
            q = nl ? nl + 1 : end;
        }
        runs.push_back({p, q});
        p = q;
    }
    return runs;
}

}  // namespace

bool LoadObj(ObjData* out, std::string* err, const char* filename, const char* mtl_basedir) {
    *out = ObjData();
    std::string buf;
    if (!read_lines(filename, &buf)) {
        if (err) *err = std::string("Cannot open file [") + filename + "]";
        return false;
    }
    const auto spans = split_runs(buf);
    std::vector<Run> runs(spans.size());
    parallel_ranges_indexed(spans.size(), [&](size_t, size_t b, size_t e) {
        for (size_t k = b; k < e; ++k) parse_run(spans[k].first, spans[k].second, &runs[k]);
    }, 1);
    // join in file order: the usemtl / mtllib lines in sequence (mtllib loads materials that later usemtl lines look up),
    // then each run's vertices and triangles
    std::unordered_map<std::string, int> mat_map;
    int cur_mat = -1;
    size_t n_vert = 0, n_tri = 0;
    std::vector<std::vector<int32_t>> mat_after(runs.size());
    for (size_t k = 0; k < runs.size(); ++k) {
        const Run& R = runs[k];
        if (R.zero_index) {
            if (err) *err = "zero face index";
            return false;
        }
        auto& ma = mat_after[k];
        ma.push_back(cur_mat);
        for (const Event& ev : R.events) {
            if (ev.mtllib) {
                Tok t{ev.text.data(), ev.text.data() + ev.text.size()};
                const char *fb, *fe;
                while (t.next(&fb, &fe)) {
                    std::string path = std::string(mtl_basedir ? mtl_basedir : "") + std::string(fb, fe);
                    if (load_mtl(path, &out->materials, &mat_map)) break;
                }
            } else {
                auto it = mat_map.find(ev.text);
                cur_mat = (it != mat_map.end()) ? it->second : -1;
            }
            ma.push_back(cur_mat);
        }
        n_vert += R.vertices.size();
        n_tri += R.tri_event.size();
    }
    std::string().swap(buf);   // the runs own everything they parsed: the file's bytes go before the outputs come
    out->vertices.resize(n_vert);
    out->triIndices.resize(3 * n_tri);
    out->triMaterial.resize(n_tri);
    std::vector<size_t> vb(runs.size() + 1, 0), tb(runs.size() + 1, 0);   // each run's first float / triangle
    for (size_t k = 0; k < runs.size(); ++k) {
        vb[k + 1] = vb[k] + runs[k].vertices.size();
        tb[k + 1] = tb[k] + runs[k].tri_event.size();
    }
    parallel_ranges_indexed(runs.size(), [&](size_t, size_t b, size_t e) {
        for (size_t k = b; k < e; ++k) {
            Run& R = runs[k];
            std::copy(R.vertices.begin(), R.vertices.end(), out->vertices.begin() + vb[k]);
            const int32_t vbase = (int32_t)(vb[k] / 3);
            for (size_t i = 0; i < R.tri.size(); ++i) out->triIndices[3 * tb[k] + i] = R.rel[i] ? vbase + R.tri[i] : R.tri[i];
            for (size_t i = 0; i < R.tri_event.size(); ++i) out->triMaterial[tb[k] + i] = mat_after[k][R.tri_event[i]];
            Run().swap_into(&R);   // each run's memory goes as soon as it is copied, so the peak is ~ the output
        }
    }, 1);
    return true;
}

}  // namespace CRT
