// pg_assets.cpp -- the atlas loader behind libenv_make (see pg_assets.h).
//
// Packs are NumPy .npz files (zip archives of .npy arrays, deflate-compressed, as written by
// tools/make_asset_pack.py); member "<dir>|<file>.png.npy" is the Qt-decoded image
// <dir>/<file>.png as uint32 [h][w] (premultiplied ARGB32 sprites, RGB32 backgrounds:
// resources.cpp:964, 969).  Decoded images are cached for the life of the process, so a second
// libenv_make of the same games does no file work.
#include "pg_assets.h"

#include <dlfcn.h>
#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>

namespace {

struct NpyArray {
    std::string descr;           // e.g. "<u4"
    std::vector<int64_t> shape;
    std::vector<uint8_t> data;   // raw little-endian elements, C order
};

struct ZipEntry {
    uint16_t method = 0;
    uint64_t csize = 0, usize = 0, local_offset = 0;
};

struct ZipFile {
    std::vector<uint8_t> bytes;
    std::map<std::string, ZipEntry> entries;
};

uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
uint64_t rd64(const uint8_t *p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

bool read_file(const std::string &path, std::vector<uint8_t> *out, std::string *err) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) {
        *err = "cannot open " + path;
        return false;
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    out->resize(n > 0 ? (size_t)n : 0);
    size_t got = n > 0 ? fread(out->data(), 1, (size_t)n, f) : 0;
    fclose(f);
    if (got != out->size()) {
        *err = "short read of " + path;
        return false;
    }
    return true;
}

// Central directory of a zip archive (with the zip64 records numpy writes for large members).
bool zip_open(const std::string &path, ZipFile *z, std::string *err) {
    if (!read_file(path, &z->bytes, err)) return false;
    const std::vector<uint8_t> &b = z->bytes;
    const size_t n = b.size();
    if (n < 22) {
        *err = path + ": not a zip archive";
        return false;
    }
    size_t eocd = std::string::npos;
    for (size_t i = n - 22 + 1; i-- > 0 && n - i <= 22 + 65535;)
        if (rd32(&b[i]) == 0x06054b50u) {
            eocd = i;
            break;
        }
    if (eocd == std::string::npos) {
        *err = path + ": no end-of-central-directory record";
        return false;
    }
    uint64_t count = rd16(&b[eocd + 10]), cd_off = rd32(&b[eocd + 16]);
    if ((count == 0xFFFF || cd_off == 0xFFFFFFFFu) && eocd >= 20 && rd32(&b[eocd - 20]) == 0x07064b50u) {
        uint64_t z64 = rd64(&b[eocd - 20 + 8]);
        if (z64 + 56 > n || rd32(&b[z64]) != 0x06064b50u) {
            *err = path + ": bad zip64 end record";
            return false;
        }
        count = rd64(&b[z64 + 32]);
        cd_off = rd64(&b[z64 + 48]);
    }
    size_t p = (size_t)cd_off;
    for (uint64_t k = 0; k < count; k++) {
        if (p + 46 > n || rd32(&b[p]) != 0x02014b50u) {
            *err = path + ": bad central directory";
            return false;
        }
        ZipEntry e;
        e.method = rd16(&b[p + 10]);
        e.csize = rd32(&b[p + 20]);
        e.usize = rd32(&b[p + 24]);
        uint16_t nl = rd16(&b[p + 28]), xl = rd16(&b[p + 30]), cl = rd16(&b[p + 32]);
        e.local_offset = rd32(&b[p + 42]);
        if (p + 46 + nl + xl + cl > n) {
            *err = path + ": truncated central directory";
            return false;
        }
        std::string name((const char *)&b[p + 46], nl);
        // zip64 extended information (header id 1): present fields in order usize, csize, offset
        for (size_t x = p + 46 + nl; x + 4 <= p + 46 + nl + xl;) {
            uint16_t id = rd16(&b[x]), len = rd16(&b[x + 2]);
            if (id == 1) {
                size_t q = x + 4;
                const size_t qend = x + 4 + len; // every 8-byte field must lie inside this record
                if (qend > p + 46 + nl + xl) {
                    *err = path + ": truncated zip64 extra field";
                    return false;
                }
                if (e.usize == 0xFFFFFFFFu) {
                    if (q + 8 > qend) { *err = path + ": short zip64 extra field"; return false; }
                    e.usize = rd64(&b[q]); q += 8;
                }
                if (e.csize == 0xFFFFFFFFu) {
                    if (q + 8 > qend) { *err = path + ": short zip64 extra field"; return false; }
                    e.csize = rd64(&b[q]); q += 8;
                }
                if (e.local_offset == 0xFFFFFFFFu) {
                    if (q + 8 > qend) { *err = path + ": short zip64 extra field"; return false; }
                    e.local_offset = rd64(&b[q]);
                }
            }
            x += 4 + len;
        }
        z->entries[name] = e;
        p += 46 + nl + xl + cl;
    }
    return true;
}

bool zip_read(const ZipFile &z, const std::string &member, const std::string &path, std::vector<uint8_t> *out,
              std::string *err) {
    auto it = z.entries.find(member);
    if (it == z.entries.end()) {
        *err = path + ": no member " + member;
        return false;
    }
    const ZipEntry &e = it->second;
    const std::vector<uint8_t> &b = z.bytes;
    if (e.local_offset + 30 > b.size() || rd32(&b[e.local_offset]) != 0x04034b50u) {
        *err = path + ": bad local header for " + member;
        return false;
    }
    size_t data = (size_t)e.local_offset + 30 + rd16(&b[e.local_offset + 26]) + rd16(&b[e.local_offset + 28]);
    if (data + e.csize > b.size()) {
        *err = path + ": truncated member " + member;
        return false;
    }
    out->resize((size_t)e.usize);
    if (e.method == 0) {
        if (e.csize != e.usize) {
            *err = path + ": stored member size mismatch";
            return false;
        }
        memcpy(out->data(), &b[data], (size_t)e.usize);
        return true;
    }
    if (e.method != 8) {
        *err = path + ": unsupported compression method for " + member;
        return false;
    }
    z_stream s;
    memset(&s, 0, sizeof(s));
    if (inflateInit2(&s, -15) != Z_OK) {
        *err = "inflateInit2 failed";
        return false;
    }
    s.next_in = const_cast<Bytef *>(&b[data]);
    s.avail_in = (uInt)e.csize;
    s.next_out = out->data();
    s.avail_out = (uInt)e.usize;
    int rc = inflate(&s, Z_FINISH);
    inflateEnd(&s);
    if (rc != Z_STREAM_END || s.total_out != e.usize) {
        *err = path + ": inflate failed for " + member;
        return false;
    }
    return true;
}

// .npy v1/v2/v3 header: "{'descr': '<u4', 'fortran_order': False, 'shape': (h, w), }"
bool npy_parse(const std::vector<uint8_t> &raw, const std::string &what, NpyArray *a, std::string *err) {
    if (raw.size() < 10 || memcmp(raw.data(), "\x93NUMPY", 6) != 0) {
        *err = what + ": not an .npy array";
        return false;
    }
    size_t hl, hs;
    if (raw[6] == 1) {
        hl = rd16(&raw[8]);
        hs = 10;
    } else {
        hl = rd32(&raw[8]);
        hs = 12;
    }
    if (hs + hl > raw.size()) {
        *err = what + ": truncated .npy header";
        return false;
    }
    std::string h((const char *)&raw[hs], hl);
    size_t d = h.find("'descr':"), f = h.find("'fortran_order':"), s = h.find("'shape':");
    if (d == std::string::npos || f == std::string::npos || s == std::string::npos) {
        *err = what + ": malformed .npy header";
        return false;
    }
    size_t q0 = h.find('\'', d + 8), q1 = q0 == std::string::npos ? q0 : h.find('\'', q0 + 1);
    const size_t fo = h.find_first_not_of(' ', f + 16);
    if (q1 == std::string::npos || fo == std::string::npos) {
        *err = what + ": malformed .npy header";
        return false;
    }
    a->descr = h.substr(q0 + 1, q1 - q0 - 1);
    if (h.compare(fo, 5, "False") != 0) {
        *err = what + ": fortran-order arrays are not supported";
        return false;
    }
    size_t p0 = h.find('(', s), p1 = p0 == std::string::npos ? p0 : h.find(')', p0);
    if (p1 == std::string::npos) {
        *err = what + ": malformed .npy shape";
        return false;
    }
    std::string dims = h.substr(p0 + 1, p1 - p0 - 1);
    a->shape.clear();
    std::stringstream ss(dims);
    std::string tok;
    while (std::getline(ss, tok, ','))
        if (tok.find_first_not_of(' ') != std::string::npos) a->shape.push_back(std::stoll(tok));
    size_t elem = a->descr.size() >= 3 ? (size_t)std::stoi(a->descr.substr(2)) : 0;
    if ((a->descr[0] != '<' && a->descr[0] != '|') || elem == 0) {
        *err = what + ": unsupported dtype " + a->descr;
        return false;
    }
    size_t count = 1;
    for (int64_t x : a->shape) count *= (size_t)x;
    if (hs + hl + count * elem != raw.size()) {
        *err = what + ": data size does not match the header";
        return false;
    }
    a->data.assign(raw.begin() + hs + hl, raw.end());
    return true;
}

std::mutex g_mu;
std::map<std::string, std::shared_ptr<ZipFile>> g_zips;              // path -> archive bytes
std::map<std::string, std::shared_ptr<const NpyArray>> g_arrays;     // path|member -> array

std::shared_ptr<const NpyArray> load_array(const std::string &path, const std::string &member, std::string *err) {
    std::lock_guard<std::mutex> lock(g_mu);
    std::string key = path + "|" + member;
    auto hit = g_arrays.find(key);
    if (hit != g_arrays.end()) return hit->second;
    auto zi = g_zips.find(path);
    std::shared_ptr<ZipFile> z;
    if (zi == g_zips.end()) {
        z = std::make_shared<ZipFile>();
        if (!zip_open(path, z.get(), err)) return nullptr;
        g_zips[path] = z;
    } else {
        z = zi->second;
    }
    std::vector<uint8_t> raw;
    if (!zip_read(*z, member + ".npy", path, &raw, err)) return nullptr;
    auto a = std::make_shared<NpyArray>();
    if (!npy_parse(raw, path + ":" + member, a.get(), err)) return nullptr;
    g_arrays[key] = a;
    return a;
}

// An image of a pack: the .npz member of key "dir/file.png" is "dir|file.png".
std::shared_ptr<const NpyArray> load_image(const std::string &path, std::string key, std::string *err) {
    for (char &c : key)
        if (c == '/') c = '|';
    auto a = load_array(path, key, err);
    if (a && (a->descr != "<u4" || a->shape.size() != 2)) {
        *err = path + ":" + key + ": expected a uint32 [h][w] image";
        return nullptr;
    }
    return a;
}

// jumper's compass overlay table (procgen_amd/assets.py compass_table_words): magic, NY, NX, MAXW,
// MAXH; per cfg x1, y1, bx0, by0, bnx, bny (int32) + cx, cy, cr (float bits); dial[4][64],
// needle[4][NY][NX][64], jump[MAXW + 1][MAXH + 1][64] as little-endian u64 -> 2 words each.
bool compass_words(const std::string &path, std::vector<uint32_t> *out, std::string *err) {
    auto geom = load_array(path, "cfg_geom", err), cf = geom ? load_array(path, "cfg_cf", err) : nullptr;
    auto dial = cf ? load_array(path, "dial", err) : nullptr, needle = dial ? load_array(path, "needle", err) : nullptr;
    auto jump = needle ? load_array(path, "jump", err) : nullptr;
    if (!jump) return false;
    if (geom->descr != "<i4" || cf->descr != "<f4" || geom->shape.size() != 2 || cf->shape.size() != 2 ||
        geom->shape[0] != cf->shape[0] || needle->shape.size() != 4 || jump->shape.size() != 3 ||
        dial->descr != "<u8" || needle->descr != "<u8" || jump->descr != "<u8") {
        *err = path + ": unexpected compass table layout";
        return false;
    }
    out->clear();
    out->push_back(0x434D5053u);
    out->push_back((uint32_t)needle->shape[1]);
    out->push_back((uint32_t)needle->shape[2]);
    out->push_back((uint32_t)(jump->shape[0] - 1));
    out->push_back((uint32_t)(jump->shape[1] - 1));
    const size_t rows = (size_t)geom->shape[0], gc = (size_t)geom->shape[1], fc = (size_t)cf->shape[1];
    for (size_t r = 0; r < rows; r++) {
        for (size_t c = 0; c < gc; c++) out->push_back(rd32(&geom->data[(r * gc + c) * 4]));
        for (size_t c = 0; c < fc; c++) out->push_back(rd32(&cf->data[(r * fc + c) * 4]));
    }
    for (const auto &a : {dial, needle, jump})
        for (size_t i = 0; i + 4 <= a->data.size(); i += 4) out->push_back(rd32(&a->data[i]));
    return true;
}

} // namespace

std::string pg_default_asset_root() {
    Dl_info info;
    if (dladdr((void *)&pg_default_asset_root, &info) && info.dli_fname) {
        std::string so(info.dli_fname);
        size_t slash = so.rfind('/');
        std::string dir = slash == std::string::npos ? std::string(".") : so.substr(0, slash);
        return dir + "/../assets";
    }
    return "assets";
}

static bool atlas_load(const std::string &root, const std::vector<int> &games, PGAtlasHost *out, std::string *err);

// The C ABI callers (libenv_make, procgen_atlas_host) must never see a C++ exception: a corrupt
// pack (a malformed number in an .npy header, an allocation failure) becomes an error message.
bool pg_atlas_load(const std::string &root, const std::vector<int> &games, PGAtlasHost *out, std::string *err) {
    try {
        return atlas_load(root, games, out, err);
    } catch (const std::exception &e) {
        *err = std::string("asset load failed: ") + e.what();
    } catch (...) {
        *err = "asset load failed";
    }
    return false;
}

static bool atlas_load(const std::string &root, const std::vector<int> &games, PGAtlasHost *out, std::string *err) {
    const int NG = 16, SLOTS = 1000, MAXBG = 64;
    out->pixels.clear();
    out->sprites.assign((size_t)NG * SLOTS * 4, 0);
    out->backgrounds.assign((size_t)NG * MAXBG * 4, 0);
    out->num_backgrounds.assign(NG, 0);
    out->num_themes.assign((size_t)NG * 100, 0);
    std::vector<uint8_t> text;
    if (!read_file(root + "/manifest.txt", &text, err)) {
        *err += " (asset manifest; set the resource_root option to the directory of the asset packs)";
        return false;
    }
    std::vector<bool> want(NG, false);
    for (int g : games)
        if (g >= 0 && g < NG) want[g] = true;
    std::map<std::string, uint32_t> placed; // "pack|key" -> pixel offset (each image once)
    auto place = [&](const std::string &pack, const std::string &key, int32_t *rec) -> bool {
        std::string path = root + "/" + pack;
        auto it = placed.find(pack + "|" + key);
        std::shared_ptr<const NpyArray> img = load_image(path, key, err);
        if (!img) return false;
        uint32_t off;
        if (it != placed.end()) {
            off = it->second;
        } else {
            off = (uint32_t)out->pixels.size();
            size_t cnt = img->data.size() / 4;
            if (out->pixels.size() + cnt >= 0x80000000ull) {
                *err = "atlas exceeds 2^31 pixels";
                return false;
            }
            out->pixels.resize(out->pixels.size() + cnt);
            memcpy(&out->pixels[off], img->data.data(), img->data.size());
            placed[pack + "|" + key] = off;
        }
        rec[0] = (int32_t)off;
        rec[1] = (int32_t)img->shape[1];
        rec[2] = (int32_t)img->shape[0];
        rec[3] = 0;
        return true;
    };
    std::istringstream in(std::string(text.begin(), text.end()));
    std::string line, sprite_pack, bg_pack;
    int gid = -1, found = 0;
    while (std::getline(in, line)) {
        if (line.empty() || line[0] == '#') continue;
        std::istringstream ls(line);
        std::string kind;
        ls >> kind;
        if (kind == "game") {
            std::string name;
            ls >> gid >> name >> sprite_pack >> bg_pack;
            if (!ls || gid < 0 || gid >= NG) {
                *err = "manifest: bad game record: " + line;
                return false;
            }
            if (want[gid]) found++;
            continue;
        }
        if (kind == "end") {
            gid = -1;
            continue;
        }
        if (gid < 0 || !want[gid]) continue;
        int a = -1;
        std::string key;
        ls >> a;
        if (kind == "themes") {
            int cnt = -1;
            ls >> cnt;
            if (!ls || a < 0 || a >= 100) {
                *err = "manifest: bad themes record: " + line;
                return false;
            }
            out->num_themes[(size_t)gid * 100 + a] = cnt;
        } else if (kind == "sprite") {
            ls >> key;
            if (!ls || a < 0 || a >= SLOTS) {
                *err = "manifest: bad sprite record: " + line;
                return false;
            }
            if (!place(sprite_pack, key, &out->sprites[((size_t)gid * SLOTS + a) * 4])) return false;
        } else if (kind == "bg") {
            ls >> key;
            if (!ls || a < 0 || a >= MAXBG) {
                *err = "manifest: bad bg record: " + line;
                return false;
            }
            if (!place(bg_pack, key, &out->backgrounds[((size_t)gid * MAXBG + a) * 4])) return false;
            if (a + 1 > out->num_backgrounds[gid]) out->num_backgrounds[gid] = a + 1;
        } else if (kind == "table") {
            ls >> key;
            if (!ls || a < 0 || a >= SLOTS) {
                *err = "manifest: bad table record: " + line;
                return false;
            }
            std::vector<uint32_t> words;
            if (!compass_words(root + "/" + key, &words, err)) return false;
            int32_t *rec = &out->sprites[((size_t)gid * SLOTS + a) * 4];
            rec[0] = (int32_t)out->pixels.size();
            rec[1] = (int32_t)words.size();
            rec[2] = 1;
            rec[3] = 0;
            out->pixels.insert(out->pixels.end(), words.begin(), words.end());
        } else {
            *err = "manifest: unknown record: " + line;
            return false;
        }
    }
    int need = 0;
    for (int g = 0; g < NG; g++) need += want[g] ? 1 : 0;
    if (found != need) {
        *err = "manifest: a game of the batch has no asset tables";
        return false;
    }
    return true;
}
