// ObjLoader.cpp — see ObjLoader.h for the semantics restated.
#include "ObjLoader.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <unordered_map>

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
void for_each_line(const std::string& buf, F&& fn) {
    const char* p = buf.data();
    const char* end = p + buf.size();
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
    for_each_line(buf, [&](const char* b, const char* e) {
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

}  // namespace

bool LoadObj(ObjData* out, std::string* err, const char* filename, const char* mtl_basedir) {
    *out = ObjData();
    std::string buf;
    if (!read_lines(filename, &buf)) {
        if (err) *err = std::string("Cannot open file [") + filename + "]";
        return false;
    }
    std::unordered_map<std::string, int> mat_map;
    int cur_mat = -1;
    bool ok = true;
    std::vector<int32_t> face;
    for_each_line(buf, [&](const char* b, const char* e) {
        if (!ok) return;
        Tok t{b, e};
        const char *kb, *ke;
        if (!t.next(&kb, &ke) || *kb == '#') return;
        const size_t kl = (size_t)(ke - kb);
        if (kl == 1 && kb[0] == 'v') {
            out->vertices.push_back(parse_real(t));
            out->vertices.push_back(parse_real(t));
            out->vertices.push_back(parse_real(t));
        } else if (kl == 1 && kb[0] == 'f') {
            const int nv = (int)(out->vertices.size() / 3);
            face.clear();
            const char *fb, *fe;
            while (t.next(&fb, &fe)) {
                int idx = atoi(fb);
                if (idx > 0) face.push_back(idx - 1);
                else if (idx < 0) face.push_back(nv + idx);
                else { ok = false; if (err) *err = "zero face index"; return; }
            }
            if (face.size() < 3) return;
            int i0 = face[0], i1, i2 = face[1];
            for (size_t k = 2; k < face.size(); ++k) {
                i1 = i2;
                i2 = face[k];
                out->triIndices.push_back(i0);
                out->triIndices.push_back(i1);
                out->triIndices.push_back(i2);
                out->triMaterial.push_back(cur_mat);
            }
        } else if (kl == 6 && memcmp(kb, "usemtl", 6) == 0) {
            t.skip();
            std::string name(t.p, t.end);
            while (!name.empty() && is_space(name.back())) name.pop_back();
            auto it = mat_map.find(name);
            cur_mat = (it != mat_map.end()) ? it->second : -1;
        } else if (kl == 6 && memcmp(kb, "mtllib", 6) == 0) {
            const char *fb, *fe;
            while (t.next(&fb, &fe)) {
                std::string path = std::string(mtl_basedir ? mtl_basedir : "") + std::string(fb, fe);
                if (load_mtl(path, &out->materials, &mat_map)) break;
            }
        }
    });
    return ok;
}

}  // namespace CRT
