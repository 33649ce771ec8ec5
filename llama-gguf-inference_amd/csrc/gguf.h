// gguf.h — GGUF v3 reader (mmap) for the llmi loader.
//
// Replaces upstream gguf_init_from_file / llama_model_loader,
// reached in the reference through `-m $MODEL` (scripts/start.sh:474).  Format per
// header, typed key/value metadata, tensor infos, data section
// aligned to general.alignment (default 32).  Tensor data stays in the read-only
// mapping; the loader streams it to HBM.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace llmi {

enum GgufType : int {
    G_U8 = 0, G_I8, G_U16, G_I16, G_U32, G_I32, G_F32, G_BOOL, G_STR, G_ARR, G_U64, G_I64, G_F64
};

struct GgufKV {
    int type = -1;
    double num = 0;          // scalar value (numeric and bool)
    std::string str;         // G_STR
    int arr_type = -1;       // G_ARR element type
    uint64_t arr_n = 0;
    std::vector<std::string> arr_str;  // G_ARR of strings
    std::vector<double> arr_num;       // G_ARR of numbers
};

struct GgufTensor {
    std::string name;
    int type = -1;
    int n_dims = 0;
    int64_t ne[4] = {1, 1, 1, 1};
    uint64_t offset = 0;
    const uint8_t* data = nullptr;
    size_t nbytes = 0;
};

class GgufFile {
public:
    GgufFile() = default;
    ~GgufFile();
    GgufFile(const GgufFile&) = delete;
    GgufFile& operator=(const GgufFile&) = delete;

    // false + err on failure
    bool open(const std::string& path, std::string& err);

    const GgufTensor* tensor(const std::string& name) const;
    const GgufKV* kv(const std::string& key) const;
    double num(const std::string& key, double dflt) const;
    std::string str(const std::string& key, const std::string& dflt) const;

    uint32_t version = 0;
    uint64_t alignment = 32;
    size_t data_start = 0;
    size_t file_size = 0;
    std::vector<GgufTensor> tensors;
    std::map<std::string, GgufKV> kvs;
    const uint8_t* map = nullptr;

private:
    int fd_ = -1;
    std::map<std::string, size_t> index_;
};

}  // namespace llmi
