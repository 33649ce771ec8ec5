// gguf.cpp — GGUF v3 reader (see gguf.h).
#include "gguf.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>

#include "common.h"

namespace llmi {

namespace {

struct Reader {
    const uint8_t* p;
    const uint8_t* end;
    bool ok = true;
    uint64_t u(int n) {
        if (!ok || end - p < n) { ok = false; return 0; }
        uint64_t v = 0;
        for (int i = 0; i < n; ++i) v |= (uint64_t)p[i] << (8 * i);
        p += n;
        return v;
    }
    std::string s() {
        uint64_t n = u(8);
        if (!ok || (uint64_t)(end - p) < n) { ok = false; return {}; }
        std::string r((const char*)p, (size_t)n);
        p += n;
        return r;
    }
};

int scalar_size(int t) {
    switch (t) {
        case G_U8: case G_I8: case G_BOOL: return 1;
        case G_U16: case G_I16: return 2;
        case G_U32: case G_I32: case G_F32: return 4;
        case G_U64: case G_I64: case G_F64: return 8;
        default: return 0;
    }
}

double scalar(Reader& r, int t) {
    uint64_t v = r.u(scalar_size(t));
    switch (t) {
        case G_I8: return (double)(int8_t)v;
        case G_I16: return (double)(int16_t)v;
        case G_I32: return (double)(int32_t)v;
        case G_I64: return (double)(int64_t)v;
        case G_F32: { uint32_t w = (uint32_t)v; float f; std::memcpy(&f, &w, 4); return f; }
        case G_F64: { double d; std::memcpy(&d, &v, 8); return d; }
        default: return (double)v;
    }
}

}  // namespace

GgufFile::~GgufFile() {
    if (map) munmap(const_cast<uint8_t*>(map), file_size);
    if (fd_ >= 0) close(fd_);
}

bool GgufFile::open(const std::string& path, std::string& err) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) { err = "cannot open " + path; return false; }
    struct stat st;
    if (fstat(fd_, &st) != 0) { err = "stat failed"; return false; }
    file_size = (size_t)st.st_size;
    if (file_size < 24) { err = "file too small for GGUF"; return false; }
    void* m = mmap(nullptr, file_size, PROT_READ, MAP_SHARED, fd_, 0);
    if (m == MAP_FAILED) { err = "mmap failed"; return false; }
    map = (const uint8_t*)m;
    Reader r{map, map + file_size};
    if (r.u(4) != 0x46554747u) { err = "bad GGUF magic"; return false; }
    version = (uint32_t)r.u(4);
    if (version != 3) { err = "unsupported GGUF version " + std::to_string(version); return false; }
    uint64_t n_tensors = r.u(8), n_kv = r.u(8);
    if (n_tensors > (1u << 24) || n_kv > (1u << 24)) { err = "implausible tensor/kv count"; return false; }
    for (uint64_t i = 0; i < n_kv && r.ok; ++i) {
        std::string key = r.s();
        GgufKV v;
        v.type = (int)r.u(4);
        if (v.type == G_STR) {
            v.str = r.s();
        } else if (v.type == G_ARR) {
            v.arr_type = (int)r.u(4);
            v.arr_n = r.u(8);
            if (v.arr_type == G_STR) {
                v.arr_str.reserve((size_t)std::min<uint64_t>(v.arr_n, 1u << 22));
                for (uint64_t k = 0; k < v.arr_n && r.ok; ++k) v.arr_str.push_back(r.s());
            } else if (scalar_size(v.arr_type) > 0) {
                if ((uint64_t)(r.end - r.p) < v.arr_n * (uint64_t)scalar_size(v.arr_type)) { r.ok = false; break; }
                v.arr_num.reserve((size_t)v.arr_n);
                for (uint64_t k = 0; k < v.arr_n && r.ok; ++k) v.arr_num.push_back(scalar(r, v.arr_type));
            } else {
                err = "unsupported nested array in " + key;
                return false;
            }
        } else if (scalar_size(v.type) > 0) {
            v.num = scalar(r, v.type);
        } else {
            err = "bad kv type for " + key;
            return false;
        }
        kvs[key] = std::move(v);
    }
    if (!r.ok) { err = "truncated GGUF metadata"; return false; }
    alignment = (uint64_t)num("general.alignment", 32);
    if (alignment == 0 || (alignment & (alignment - 1))) { err = "bad general.alignment"; return false; }
    tensors.resize((size_t)n_tensors);
    for (uint64_t i = 0; i < n_tensors && r.ok; ++i) {
        GgufTensor& t = tensors[i];
        t.name = r.s();
        t.n_dims = (int)r.u(4);
        if (t.n_dims < 1 || t.n_dims > 4) { err = "bad n_dims for " + t.name; return false; }
        for (int d = 0; d < t.n_dims; ++d) t.ne[d] = (int64_t)r.u(8);
        t.type = (int)r.u(4);
        t.offset = r.u(8);
    }
    if (!r.ok) { err = "truncated GGUF tensor infos"; return false; }
    data_start = align_up((size_t)(r.p - map), alignment);
    for (size_t i = 0; i < tensors.size(); ++i) {
        GgufTensor& t = tensors[i];
        if (!type_supported(t.type)) { err = "tensor " + t.name + ": unsupported ggml type " + std::to_string(t.type); return false; }
        // upstream gguf_init_from_file rejects negative dims and element counts past
        // INT64_MAX; every product and the end offset are computed overflow-checked
        int64_t n = 1;
        for (int d = 0; d < 4; ++d) {
            if (t.ne[d] < 0) { err = "tensor " + t.name + ": negative dimension"; return false; }
            if (t.ne[d] != 0 && n > INT64_MAX / t.ne[d]) { err = "tensor " + t.name + ": element count overflows"; return false; }
            n *= t.ne[d];
        }
        if (t.ne[0] == 0 || t.ne[0] % block_elems(t.type)) { err = "tensor " + t.name + ": row not a whole number of blocks"; return false; }
        const uint64_t nblk = (uint64_t)(n / block_elems(t.type));
        if (nblk > (uint64_t)file_size / (uint64_t)block_bytes(t.type)) { err = "tensor " + t.name + " extends past end of file"; return false; }
        t.nbytes = (size_t)nblk * (size_t)block_bytes(t.type);
        if (t.offset % alignment) { err = "tensor " + t.name + ": misaligned offset"; return false; }
        if (t.offset > file_size || data_start > file_size - t.offset || t.nbytes > file_size - data_start - t.offset) {
            err = "tensor " + t.name + " extends past end of file";
            return false;
        }
        t.data = map + data_start + t.offset;
        index_[t.name] = i;
    }
    return true;
}

const GgufTensor* GgufFile::tensor(const std::string& name) const {
    auto it = index_.find(name);
    return it == index_.end() ? nullptr : &tensors[it->second];
}
const GgufKV* GgufFile::kv(const std::string& key) const {
    auto it = kvs.find(key);
    return it == kvs.end() ? nullptr : &it->second;
}
double GgufFile::num(const std::string& key, double dflt) const {
    const GgufKV* v = kv(key);
    return (v && v->type != G_STR && v->type != G_ARR) ? v->num : dflt;
}
std::string GgufFile::str(const std::string& key, const std::string& dflt) const {
    const GgufKV* v = kv(key);
    return (v && v->type == G_STR) ? v->str : dflt;
}

}  // namespace llmi
