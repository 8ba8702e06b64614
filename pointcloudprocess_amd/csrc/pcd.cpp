// PCD v0.7 I/O of PointXYZRGBA clouds: the on-disk format of every
// hot-path input (io::loadPCDFile, main_blend.cpp:343-351, 456, 533, 763, 1013) and output
// (io::savePCDFile / savePCDFileBinary, main_blend.cpp:839-916), host-only, reading into and
// writing from caller buffers (pinned host memory stages straight to the device).
//   pcp_pcd_write  PCDWriter::generateHeader + writeBinary / writeBinaryCompressed
//                  (pcd_helper.h:321-371, 489-610, 628-790): fields x y z rgba stamp_id
//                  (point_type.h:326-332), point-major packed records, or SoA planes + LZF
//   pcp_pcd_read   PCDReader::read (pcd_helper.cpp:71-1395) for DATA ascii / binary /
//                  binary_compressed with any field subset and order; fields absent from the
//                  file keep PointXYZRGBA's defaults (x = y = z = 0, data[3] = 1, rgba = 0)
//   pcp_lzf_*      the LZF codec of lzf.cpp:86-415 (HLOG 13 hash, 8 KB window, literal runs of
//                  up to 32, back references of up to 264): same compressed bytes
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pcp.h"

namespace {

constexpr int kHlog = 13;
inline uint32_t lzf_slot(uint32_t h) { return ((h >> (3 * 8 - kHlog)) - h) & ((1u << kHlog) - 1); }

// The compressor walks the input with a 3-byte rolling hash into a table of last positions;
// a candidate at distance <= 8192 whose first 3 bytes match (never at position 0: the table's
// empty value) is extended to at most 264 bytes and emitted as a back reference, otherwise the
// byte joins the current literal run.  Returns 0 when the output does not fit.
size_t lzf_compress(const uint8_t* in, size_t in_len, uint8_t* out, size_t out_len) {
    if (!in_len || !out_len) return 0;
    std::vector<uint32_t> htab((size_t)1 << kHlog, 0u);
    const uint8_t* ip = in;
    const uint8_t* const in_end = in + in_len;
    uint8_t* op = out;
    uint8_t* const out_end = out + out_len;
    int lit = 0;
    op++;  // the first literal run's control byte
    uint32_t hval = in_len >= 2 ? ((uint32_t)ip[0] << 8) | ip[1] : 0u;
    while (in_len >= 3 && ip < in_end - 2) {
        hval = (hval << 8) | ip[2];
        uint32_t* hs = &htab[lzf_slot(hval)];
        const uint8_t* ref = in + *hs;
        *hs = (uint32_t)(ip - in);
        size_t off;
        if (ref < ip && (off = (size_t)(ip - ref - 1)) < ((size_t)1 << 13) && ref > in && ref[2] == ip[2] &&
            ref[0] == ip[0] && ref[1] == ip[1]) {
            size_t len = 2;
            size_t maxlen = (size_t)(in_end - ip) - len;
            if (maxlen > (1u << 8) + (1u << 3)) maxlen = (1u << 8) + (1u << 3);
            if (op + 3 + 1 >= out_end && op - !lit + 3 + 1 >= out_end) return 0;
            op[-lit - 1] = (uint8_t)(lit - 1);  // close the literal run
            op -= !lit;                          // (or drop its empty control byte)
            // extend: with maxlen > 16 the first 16 steps do not test maxlen (lzf.cpp:145-203), so a
            // run reaching the input's end can exceed maxlen by up to 2 -- kept, it is the format
            bool stop = false;
            if (maxlen > 16) {
                for (int u = 0; u < 16 && !stop; u++) {
                    len++;
                    stop = ref[len] != ip[len];
                }
            }
            if (!stop) {
                do {
                    len++;
                } while (len < maxlen && ref[len] == ip[len]);
            }
            len -= 2;  // octets - 1 ... encoded as len - 2 + 2
            ip++;
            if (len < 7) {
                *op++ = (uint8_t)((off >> 8) + (len << 5));
            } else {
                *op++ = (uint8_t)((off >> 8) + (7 << 5));
                *op++ = (uint8_t)(len - 7);
            }
            *op++ = (uint8_t)off;
            lit = 0;
            op++;
            ip += len + 1;
            if (ip >= in_end - 2) break;
            --ip;
            hval = ((uint32_t)ip[0] << 8) | ip[1];
            hval = (hval << 8) | ip[2];
            htab[lzf_slot(hval)] = (uint32_t)(ip - in);
            ip++;
        } else {
            if (op >= out_end) return 0;
            lit++;
            *op++ = *ip++;
            if (lit == 32) {
                op[-lit - 1] = (uint8_t)(lit - 1);
                lit = 0;
                op++;
            }
        }
    }
    if (op + 3 > out_end) return 0;
    while (ip < in_end) {
        lit++;
        *op++ = *ip++;
        if (lit == 32) {
            op[-lit - 1] = (uint8_t)(lit - 1);
            lit = 0;
            op++;
        }
    }
    op[-lit - 1] = (uint8_t)(lit - 1);
    op -= !lit;
    return (size_t)(op - out);
}

size_t lzf_decompress(const uint8_t* in, size_t in_len, uint8_t* out, size_t out_len) {
    const uint8_t* ip = in;
    const uint8_t* const in_end = in + in_len;
    uint8_t* op = out;
    uint8_t* const out_end = out + out_len;
    while (ip < in_end) {
        uint32_t ctrl = *ip++;
        if (ctrl < 32) {  // literal run of ctrl + 1 octets
            ctrl++;
            if (op + ctrl > out_end || ip + ctrl > in_end) return 0;
            std::memcpy(op, ip, ctrl);
            op += ctrl;
            ip += ctrl;
        } else {  // back reference: length (ctrl >> 5) + 2, offset ((ctrl & 31) << 8 | next) + 1
            size_t len = ctrl >> 5;
            if (ip >= in_end) return 0;
            if (len == 7) {
                len += *ip++;
                if (ip >= in_end) return 0;
            }
            const uint8_t* ref = op - ((ctrl & 0x1f) << 8) - 1 - *ip++;
            len += 2;
            if (op + len > out_end || ref < out) return 0;
            for (size_t k = 0; k < len; k++) op[k] = ref[k];  // may overlap: byte order
            op += len;
        }
    }
    return (size_t)(op - out);
}

struct Field {
    std::string name;
    int size = 0, count = 1;
    char type = 'F';
};

// header tokens of one line
std::vector<std::string> split(const std::string& s) {
    std::vector<std::string> t;
    size_t i = 0;
    while (i < s.size()) {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\r')) i++;
        size_t j = i;
        while (j < s.size() && s[j] != ' ' && s[j] != '\t' && s[j] != '\r') j++;
        if (j > i) t.push_back(s.substr(i, j - i));
        i = j;
    }
    return t;
}

struct Layout {  // where a file field lands in the 48-byte record
    int dst = -1;  // 0..2: x, y, z (double); 3: rgba; 4: stamp_id
};

double as_double(const uint8_t* p, const Field& f) {
    switch (f.type) {
        case 'F': {
            if (f.size == 8) { double v; std::memcpy(&v, p, 8); return v; }
            float v; std::memcpy(&v, p, 4); return v;
        }
        case 'U': {
            if (f.size == 1) return *p;
            if (f.size == 2) { uint16_t v; std::memcpy(&v, p, 2); return v; }
            uint32_t v; std::memcpy(&v, p, 4); return v;
        }
        default: {
            if (f.size == 1) return (int8_t)*p;
            if (f.size == 2) { int16_t v; std::memcpy(&v, p, 2); return v; }
            int32_t v; std::memcpy(&v, p, 4); return v;
        }
    }
}
uint32_t as_bits32(const uint8_t* p, const Field& f) {
    if (f.size == 4) { uint32_t v; std::memcpy(&v, p, 4); return v; }  // rgb as packed float: its bits
    return (uint32_t)as_double(p, f);
}

void put(uint8_t* rec, const Layout& l, const uint8_t* src, const Field& f) {
    if (l.dst < 0) return;
    if (l.dst < 3) {
        const double v = as_double(src, f);
        std::memcpy(rec + 8 * l.dst, &v, 8);
    } else {
        const uint32_t v = as_bits32(src, f);
        std::memcpy(rec + (l.dst == 3 ? 32 : 36), &v, 4);
    }
}

void default_record(uint8_t* rec) {  // PointXYZRGBA() (point_type.h:86-91)
    std::memset(rec, 0, 48);
    const double one = 1.0;
    std::memcpy(rec + 24, &one, 8);
}

}  // namespace

extern "C" {

size_t pcp_lzf_compress(const void* in, size_t in_len, void* out, size_t out_len) {
    return lzf_compress((const uint8_t*)in, in_len, (uint8_t*)out, out_len);
}
size_t pcp_lzf_decompress(const void* in, size_t in_len, void* out, size_t out_len) {
    return lzf_decompress((const uint8_t*)in, in_len, (uint8_t*)out, out_len);
}

int pcp_pcd_write(const char* path, const void* pts_host, int64_t n, int64_t width, int64_t height, int compressed) {
    if (!path || n < 0 || (n > 0 && !pts_host)) return PCP_ERR_ARG;
    if (n == 0) return PCP_ERR_EMPTY;  // "Input point cloud has no data!" (pcd_helper.h:492-495)
    if (width <= 0 || height <= 0) { width = n; height = 1; }
    char hdr[512];
    std::snprintf(hdr, sizeof(hdr),
                  "# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z rgba stamp_id\nSIZE 8 8 8 4 4\n"
                  "TYPE F F F U U\nCOUNT 1 1 1 1 1\nWIDTH %lld\nHEIGHT %lld\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS %lld\n"
                  "DATA %s\n",
                  (long long)width, (long long)height, (long long)n, compressed ? "binary_compressed" : "binary");
    const uint8_t* src = (const uint8_t*)pts_host;
    const size_t fsize = 32, data_size = (size_t)n * fsize;
    std::vector<uint8_t> body;
    if (!compressed) {  // point-major: x y z rgba stamp_id (writeBinary, :519-590)
        body.resize(data_size);
        for (int64_t i = 0; i < n; i++) {
            std::memcpy(&body[i * fsize], src + 48 * i, 24);
            std::memcpy(&body[i * fsize + 24], src + 48 * i + 32, 8);
        }
    } else {  // SoA planes x.. y.. z.. rgba.. stamp.. then LZF with an 8-byte size header (:666-731)
        if (data_size > 0xffffffffull) return PCP_ERR_CAPACITY;  // 32-bit size fields
        std::vector<uint8_t> planes(data_size);
        const size_t offs[5] = {0, 8, 16, 32, 36}, sizes[5] = {8, 8, 8, 4, 4};
        size_t p0 = 0;
        for (int f = 0; f < 5; f++) {
            for (int64_t i = 0; i < n; i++) std::memcpy(&planes[p0 + i * sizes[f]], src + 48 * i + offs[f], sizes[f]);
            p0 += sizes[f] * (size_t)n;
        }
        const size_t cap = (size_t)((float)data_size * 1.5f);
        body.resize(cap + 8);
        const size_t cs = lzf_compress(planes.data(), data_size, &body[8], cap);
        if (!cs) return PCP_ERR_CAPACITY;  // "Error during compression!"
        const uint32_t c32 = (uint32_t)cs, u32 = (uint32_t)data_size;
        std::memcpy(&body[0], &c32, 4);
        std::memcpy(&body[4], &u32, 4);
        body.resize(cs + 8);
    }
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return PCP_ERR_ARG;  // "Error during open!"
    const size_t hl = std::strlen(hdr);
    const bool ok = std::fwrite(hdr, 1, hl, fp) == hl && std::fwrite(body.data(), 1, body.size(), fp) == body.size();
    std::fclose(fp);
    return ok ? PCP_OK : PCP_ERR_ARG;
}

// is_dense as the reference's reader sets it (pcd_helper.cpp:863, 1124-1179): true unless a
// binary / binary_compressed field value of some point is non-finite (ascii stays dense)
static bool field_finite(const uint8_t* p, const Field& f) {
    if (f.type != 'F') return true;  // integers are always finite
    if (f.size == 8) { double v; std::memcpy(&v, p, 8); return std::isfinite(v); }
    float v; std::memcpy(&v, p, 4); return std::isfinite(v);
}

int pcp_pcd_read_ex(const char* path, void* out_host, int64_t cap, int64_t* n_out, int64_t* width_out,
                    int64_t* height_out, int* dense_out) {
    if (!path || !n_out) return PCP_ERR_ARG;
    *n_out = 0;
    if (width_out) *width_out = 0;
    if (height_out) *height_out = 0;
    if (dense_out) *dense_out = 1;
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return PCP_ERR_ARG;
    std::fseek(fp, 0, SEEK_END);
    const long fl = std::ftell(fp);
    std::fseek(fp, 0, SEEK_SET);
    std::vector<uint8_t> file(fl > 0 ? (size_t)fl : 0);
    const bool rd = file.empty() || std::fread(file.data(), 1, file.size(), fp) == file.size();
    std::fclose(fp);
    if (!rd) return PCP_ERR_ARG;
    // header: lines up to and including DATA
    std::vector<Field> fields;
    int64_t npts = -1, width = 0, height = 1;
    bool have_points = false;
    std::string data;
    size_t pos = 0;
    while (pos < file.size()) {
        size_t e = pos;
        while (e < file.size() && file[e] != '\n') e++;
        const std::string line((const char*)&file[pos], e - pos);
        pos = e < file.size() ? e + 1 : file.size();  // a last line without '\n' ends at the file's end
        const std::vector<std::string> t = split(line);
        if (t.empty() || t[0][0] == '#') continue;
        if (t[0] == "FIELDS" || t[0] == "COLUMNS") {
            fields.assign(t.size() - 1, Field());
            for (size_t k = 1; k < t.size(); k++) fields[k - 1].name = t[k];
        } else if (t[0] == "SIZE") {
            for (size_t k = 1; k < t.size() && k - 1 < fields.size(); k++) fields[k - 1].size = std::atoi(t[k].c_str());
        } else if (t[0] == "TYPE") {
            for (size_t k = 1; k < t.size() && k - 1 < fields.size(); k++) fields[k - 1].type = t[k][0];
        } else if (t[0] == "COUNT") {
            for (size_t k = 1; k < t.size() && k - 1 < fields.size(); k++) fields[k - 1].count = std::atoi(t[k].c_str());
        } else if (t[0] == "WIDTH" && t.size() > 1) {
            width = std::atoll(t[1].c_str());
        } else if (t[0] == "HEIGHT" && t.size() > 1) {
            height = std::atoll(t[1].c_str());
        } else if (t[0] == "POINTS" && t.size() > 1) {
            npts = std::atoll(t[1].c_str());
            have_points = true;
        } else if (t[0] == "DATA" && t.size() > 1) {
            data = t[1];
            break;
        }
    }
    if (data.empty() || fields.empty()) return PCP_ERR_ARG;
    if (width < 0 || height < 0 || (have_points && npts < 0)) return PCP_ERR_ARG;
    if (!have_points) {
        if (width > 0 && height > ((int64_t)1 << 62) / width) return PCP_ERR_ARG;
        npts = width * height;
    }
    // the PCL datatypes the reference's reader accepts (sensor_msgs::PointField): F 4/8, U/I 1/2/4
    size_t psize = 0;
    for (size_t f = 0; f < fields.size(); f++) {
        const char ty = fields[f].type;
        const int sz = fields[f].size;
        const bool ok = (ty == 'F' && (sz == 4 || sz == 8)) || ((ty == 'U' || ty == 'I') && (sz == 1 || sz == 2 || sz == 4));
        if (!ok) return PCP_ERR_ARG;
        if (fields[f].count < 1) fields[f].count = 1;
        if (fields[f].count > (1 << 20)) return PCP_ERR_ARG;
        psize += (size_t)sz * (size_t)fields[f].count;
    }
    *n_out = npts;
    if (width_out) *width_out = width;
    if (height_out) *height_out = height;
    if (!out_host) return PCP_OK;  // size query
    if (npts > cap) return PCP_ERR_CAPACITY;
    // bytes of point data the header promises, overflow-checked
    if (npts > 0 && psize > (SIZE_MAX / 2) / (size_t)npts) return PCP_ERR_ARG;
    const size_t need = psize * (size_t)npts;
    const size_t remain = file.size() - pos;  // pos <= file.size() by construction
    std::vector<Layout> lay(fields.size());
    for (size_t f = 0; f < fields.size(); f++) {
        const std::string& nm = fields[f].name;
        if (fields[f].count == 1) {
            if (nm == "x") lay[f].dst = 0;
            else if (nm == "y") lay[f].dst = 1;
            else if (nm == "z") lay[f].dst = 2;
            else if (nm == "rgba" || nm == "rgb") lay[f].dst = 3;
            else if (nm == "stamp_id") lay[f].dst = 4;
        }
    }
    uint8_t* out = (uint8_t*)out_host;
    for (int64_t i = 0; i < npts; i++) default_record(out + 48 * i);
    bool dense = true;
    if (data == "binary") {
        if (remain < need) return PCP_ERR_ARG;
        for (int64_t i = 0; i < npts; i++) {
            const uint8_t* row = &file[pos + psize * (size_t)i];
            size_t o = 0;
            for (size_t f = 0; f < fields.size(); f++) {
                put(out + 48 * i, lay[f], row + o, fields[f]);
                for (int c = 0; c < fields[f].count; c++) dense = dense && field_finite(row + o + (size_t)c * fields[f].size, fields[f]);
                o += (size_t)fields[f].size * fields[f].count;
            }
        }
    } else if (data == "binary_compressed") {
        if (remain < 8) return PCP_ERR_ARG;
        uint32_t csz, usz;
        std::memcpy(&csz, &file[pos], 4);
        std::memcpy(&usz, &file[pos + 4], 4);
        if (remain - 8 < csz || usz < need) return PCP_ERR_ARG;
        std::vector<uint8_t> planes(usz);
        if (lzf_decompress(&file[pos + 8], csz, planes.data(), usz) != usz) return PCP_ERR_ARG;
        size_t p0 = 0;
        for (size_t f = 0; f < fields.size(); f++) {
            const size_t fs = (size_t)fields[f].size * fields[f].count;
            for (int64_t i = 0; i < npts; i++) {
                const uint8_t* src = &planes[p0 + fs * (size_t)i];
                put(out + 48 * i, lay[f], src, fields[f]);
                for (int c = 0; c < fields[f].count; c++) dense = dense && field_finite(src + (size_t)c * fields[f].size, fields[f]);
            }
            p0 += fs * (size_t)npts;
        }
    } else if (data == "ascii") {
        const char* s = (const char*)file.data() + pos;
        const char* end = (const char*)file.data() + file.size();
        std::string tok;
        for (int64_t i = 0; i < npts; i++) {
            for (size_t f = 0; f < fields.size(); f++) {
                for (int c = 0; c < fields[f].count; c++) {
                    while (s < end && (*s == ' ' || *s == '\t' || *s == '\r' || *s == '\n')) s++;
                    const char* b = s;
                    while (s < end && !(*s == ' ' || *s == '\t' || *s == '\r' || *s == '\n')) s++;
                    if (b == s) return PCP_ERR_ARG;
                    if (c > 0 || lay[f].dst < 0) continue;
                    tok.assign(b, s - b);
                    uint8_t* rec = out + 48 * i;
                    if (lay[f].dst < 3) {
                        const double v = std::strtod(tok.c_str(), nullptr);
                        std::memcpy(rec + 8 * lay[f].dst, &v, 8);
                    } else {
                        uint32_t v;
                        if (fields[f].type == 'F') {  // a packed rgb float printed as a float
                            const float fv = std::strtof(tok.c_str(), nullptr);
                            std::memcpy(&v, &fv, 4);
                        } else {
                            v = (uint32_t)std::strtoul(tok.c_str(), nullptr, 10);
                        }
                        std::memcpy(rec + (lay[f].dst == 3 ? 32 : 36), &v, 4);
                    }
                }
            }
        }
    } else {
        return PCP_ERR_UNSUPPORTED;
    }
    if (dense_out) *dense_out = dense ? 1 : 0;
    return PCP_OK;
}

int pcp_pcd_read(const char* path, void* out_host, int64_t cap, int64_t* n_out) {
    return pcp_pcd_read_ex(path, out_host, cap, n_out, nullptr, nullptr, nullptr);
}

}  // extern "C"
