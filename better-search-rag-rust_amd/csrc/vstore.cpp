// vstore.cpp -- the reference's parquet vector store (src/vectorstore/polars.rs) read and
// written natively with Apache Arrow C++ / Parquet, and the rank's block loaded straight
// into a bsr_index.  Host-only; libbsr_vstore.so, linked to libbsr.so.
//
// Storage model: the rows read from the file stay in their Arrow chunks (zero copy); rows
// appended since (append_many) live in a dense side buffer; persist writes both as one
// "embeddings" List(Float32) column (zstd when available, as polars' default writer).
#include <arrow/api.h>
#include <arrow/io/api.h>
#include <parquet/arrow/reader.h>
#include <parquet/arrow/writer.h>
#include <parquet/properties.h>

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <filesystem>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "bsr_vstore.h"

namespace fs = std::filesystem;

namespace bsr {
int set_error(int code, const char* fmt, ...);
void clear_error();
}  // namespace bsr
using bsr::set_error;

struct bsr_vstore {
    std::string path;
    std::shared_ptr<arrow::ChunkedArray> col;  // rows read from the file (may be null)
    std::vector<float> app_vals;                // appended rows, back to back
    std::vector<uint64_t> app_off{0};           // app_off[i]..app_off[i+1]: appended row i

    uint64_t file_rows() const { return col ? (uint64_t)col->length() : 0; }
    uint64_t count() const { return file_rows() + (app_off.size() - 1); }
};

namespace {

const char* kColumn = "embeddings";  // polars.rs:17-27

#define VS_TRY(expr)                  \
    do {                              \
        int r_ = (expr);              \
        if (r_ != BSR_OK) return r_;  \
    } while (0)

int arrow_error(const arrow::Status& st, const char* what) {
    return set_error(BSR_E_INVALID, "%s: %s", what, st.ToString().c_str());
}

std::shared_ptr<arrow::DataType> list_type() { return arrow::list(arrow::field("item", arrow::float32())); }

// One row visitor over a ListArray / LargeListArray / FixedSizeListArray chunk.  Calls
// f(valid, values, value_offset, length) for row i of the chunk.
template <class F>
int visit_chunk_row(const arrow::Array& a, int64_t i, F&& f) {
    using T = arrow::Type;
    switch (a.type_id()) {
        case T::LIST: {
            const auto& l = static_cast<const arrow::ListArray&>(a);
            return f(l.IsValid(i), l.values(), (int64_t)l.value_offset(i), (int64_t)l.value_length(i));
        }
        case T::LARGE_LIST: {
            const auto& l = static_cast<const arrow::LargeListArray&>(a);
            return f(l.IsValid(i), l.values(), (int64_t)l.value_offset(i), (int64_t)l.value_length(i));
        }
        case T::FIXED_SIZE_LIST: {
            const auto& l = static_cast<const arrow::FixedSizeListArray&>(a);
            return f(l.IsValid(i), l.values(), (int64_t)l.value_offset(i), (int64_t)l.value_length(i));
        }
        default:
            return set_error(BSR_E_INVALID, "column '%s' is %s, expected List(Float32)", kColumn,
                             a.type()->ToString().c_str());
    }
}

// polars' DataFrame::slice offsets: a negative offset counts from the end, both ends are
// clamped to [0, height].
void slice_bounds(int64_t offset, uint64_t length, uint64_t height, uint64_t* start, uint64_t* stop) {
    const int64_t h = (int64_t)height;
    const int64_t s = offset < 0 ? h + offset : offset;
    const int64_t len = length > (uint64_t)INT64_MAX ? INT64_MAX : (int64_t)length;
    const int64_t e = s > INT64_MAX - len ? INT64_MAX : s + len;
    *start = (uint64_t)std::clamp<int64_t>(s, 0, h);
    *stop = (uint64_t)std::clamp<int64_t>(e, 0, h);
}

// Walk rows [start, stop) in order: row(length, copy_fn) per non-null row, where copy_fn(dst)
// writes its non-null elements.  Mirrors get_many's filter_map (null rows dropped) and
// flatten (null elements skipped).
template <class RowFn>
int walk_rows(const bsr_vstore* vs, uint64_t start, uint64_t stop, RowFn&& row) {
    uint64_t base = 0;
    if (vs->col) {
        for (const auto& chunk : vs->col->chunks()) {
            const uint64_t len = (uint64_t)chunk->length();
            const uint64_t lo = std::max(start, base), hi = std::min(stop, base + len);
            for (uint64_t g = lo; g < hi; ++g) {
                VS_TRY(visit_chunk_row(*chunk, (int64_t)(g - base),
                                       [&](bool valid, const std::shared_ptr<arrow::Array>& values, int64_t off,
                                           int64_t n) -> int {
                                           if (!valid) return BSR_OK;
                                           if (values->type_id() != arrow::Type::FLOAT)
                                               return set_error(BSR_E_INVALID, "list values are %s, expected float",
                                                                values->type()->ToString().c_str());
                                           const auto& fa = static_cast<const arrow::FloatArray&>(*values);
                                           uint32_t nn = 0;
                                           for (int64_t j = 0; j < n; ++j) nn += fa.IsValid(off + j) ? 1u : 0u;
                                           return row(nn, [&](float* dst) {
                                               for (int64_t j = 0; j < n; ++j)
                                                   if (fa.IsValid(off + j)) *dst++ = fa.Value(off + j);
                                           });
                                       }));
            }
            base += len;
            if (base >= stop) return BSR_OK;
        }
    }
    const uint64_t fr = vs->file_rows();
    for (uint64_t g = std::max(start, fr); g < stop; ++g) {
        const uint64_t a = vs->app_off[g - fr], b = vs->app_off[g - fr + 1];
        VS_TRY(row((uint32_t)(b - a),
                   [&](float* dst) { memcpy(dst, vs->app_vals.data() + a, (b - a) * sizeof(float)); }));
    }
    return BSR_OK;
}

// read_parquet (polars.rs:50-77): the file's "embeddings" column; a missing file is
// created (with its parent directories) holding an empty column.
int write_table(const std::string& path, const std::shared_ptr<arrow::Array>& arr);

int read_parquet(const std::string& path, std::shared_ptr<arrow::ChunkedArray>* out) {
    std::error_code ec;
    const fs::path p(path);
    if (!fs::exists(p, ec)) {
        if (p.has_parent_path() && !fs::exists(p.parent_path(), ec)) {
            fs::create_directories(p.parent_path(), ec);
            if (ec) return set_error(BSR_E_INVALID, "Failed to create directory: %s", ec.message().c_str());
        }
        arrow::ListBuilder b(arrow::default_memory_pool(), std::make_shared<arrow::FloatBuilder>(), list_type());
        std::shared_ptr<arrow::Array> empty;
        auto st = b.Finish(&empty);
        if (!st.ok()) return arrow_error(st, "empty column");
        VS_TRY(write_table(path, empty));
        *out = std::make_shared<arrow::ChunkedArray>(arrow::ArrayVector{empty}, list_type());
        return BSR_OK;
    }
    auto f = arrow::io::ReadableFile::Open(path);
    if (!f.ok()) return arrow_error(f.status(), "open");
    auto rd = parquet::arrow::OpenFile(*f, arrow::default_memory_pool());
    if (!rd.ok()) return arrow_error(rd.status(), "parquet open");
    auto tr = (*rd)->ReadTable();
    if (!tr.ok()) return arrow_error(tr.status(), "parquet read");
    std::shared_ptr<arrow::Table> t = *tr;
    auto c = t->GetColumnByName(kColumn);
    if (!c) return set_error(BSR_E_INVALID, "no column '%s' in %s", kColumn, path.c_str());
    *out = c;
    return BSR_OK;
}

int write_table(const std::string& path, const std::shared_ptr<arrow::Array>& arr) {
    auto schema = arrow::schema({arrow::field(kColumn, arr->type())});
    auto table = arrow::Table::Make(schema, {arr});
    auto out = arrow::io::FileOutputStream::Open(path);
    if (!out.ok()) return set_error(BSR_E_INVALID, "Error creating file: %s", out.status().ToString().c_str());
    parquet::WriterProperties::Builder pb;
    if (arrow::util::Codec::IsAvailable(arrow::Compression::ZSTD)) pb.compression(parquet::Compression::ZSTD);
    auto st = parquet::arrow::WriteTable(*table, arrow::default_memory_pool(), *out, 1 << 16, pb.build());
    if (!st.ok()) return arrow_error(st, "parquet write");
    st = (*out)->Close();
    if (!st.ok()) return arrow_error(st, "close");
    return BSR_OK;
}

int slice_sizes(const bsr_vstore* vs, uint64_t start, uint64_t stop, uint64_t* rows, uint64_t* floats) {
    *rows = 0;
    *floats = 0;
    return walk_rows(vs, start, stop, [&](uint32_t n, auto&&) -> int {
        ++*rows;
        *floats += n;
        return BSR_OK;
    });
}

}  // namespace

#define VS_GUARD(expr)                                                   \
    try {                                                                \
        bsr::clear_error();                                              \
        return (expr);                                                   \
    } catch (const std::bad_alloc&) {                                    \
        return set_error(BSR_E_NOMEM, "host allocation failed");         \
    } catch (const std::exception& e) {                                  \
        return set_error(BSR_E_INVALID, "internal error: %s", e.what()); \
    } catch (...) {                                                      \
        return set_error(BSR_E_INVALID, "internal error");               \
    }

extern "C" {

int bsr_vstore_open(const char* path, int empty, bsr_vstore** out) {
    VS_GUARD(([&]() -> int {
        if (!path || !out) return set_error(BSR_E_INVALID, "null argument");
        *out = nullptr;
        auto vs = std::make_unique<bsr_vstore>();
        vs->path = path;
        if (!empty) VS_TRY(read_parquet(vs->path, &vs->col));
        *out = vs.release();
        return BSR_OK;
    })());
}

void bsr_vstore_close(bsr_vstore* vs) { delete vs; }

const char* bsr_vstore_path(const bsr_vstore* vs) { return vs ? vs->path.c_str() : ""; }

int bsr_vstore_get_count(const bsr_vstore* vs, uint64_t* out) {
    if (!vs || !out) return set_error(BSR_E_INVALID, "null argument");
    *out = vs->count();
    return BSR_OK;
}

int bsr_vstore_get_many(const bsr_vstore* vs, int64_t offset, uint64_t length, float* out, uint64_t out_capacity,
                        uint32_t* row_len, uint64_t len_capacity, uint64_t* out_rows, uint64_t* out_floats) {
    VS_GUARD(([&]() -> int {
        if (!vs || !out_rows || !out_floats) return set_error(BSR_E_INVALID, "null argument");
        uint64_t start, stop, rows, floats;
        slice_bounds(offset, length, vs->count(), &start, &stop);
        VS_TRY(slice_sizes(vs, start, stop, &rows, &floats));
        *out_rows = rows;
        *out_floats = floats;
        if (!out && !row_len) return BSR_OK;
        if ((out && floats > out_capacity) || (row_len && rows > len_capacity))
            return set_error(BSR_E_INVALID, "output too small (%llu rows, %llu floats)", (unsigned long long)rows,
                             (unsigned long long)floats);
        uint64_t r = 0;
        float* dst = out;
        return walk_rows(vs, start, stop, [&](uint32_t n, auto&& copy) -> int {
            if (row_len) row_len[r] = n;
            if (dst) {
                copy(dst);
                dst += n;
            }
            ++r;
            return BSR_OK;
        });
    })());
}

int bsr_vstore_read_slab(const bsr_vstore* vs, int64_t offset, uint64_t length, uint32_t dim, float* out,
                         uint64_t capacity_rows, uint64_t* out_rows) {
    VS_GUARD(([&]() -> int {
        if (!vs || !out_rows || (!out && capacity_rows)) return set_error(BSR_E_INVALID, "null argument");
        uint64_t start, stop;
        slice_bounds(offset, length, vs->count(), &start, &stop);
        hipPointerAttribute_t attr;
        bool dev = false;
        if (out && hipPointerGetAttributes(&attr, out) == hipSuccess)
            dev = attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
        (void)hipGetLastError();
        std::vector<float> stage;
        uint64_t r = 0;
        VS_TRY(walk_rows(vs, start, stop, [&](uint32_t n, auto&& copy) -> int {
            if (n != dim)
                return set_error(BSR_E_DIM, "row %llu has %u elements, expected %u", (unsigned long long)(start + r), n,
                                 dim);
            if (r >= capacity_rows) return set_error(BSR_E_INVALID, "output too small");
            if (dev) {
                stage.resize(dim);
                copy(stage.data());
                if (hipMemcpy(out + r * dim, stage.data(), (size_t)dim * sizeof(float), hipMemcpyHostToDevice) !=
                    hipSuccess)
                    return set_error(BSR_E_HIP, "hipMemcpy to device failed");
            } else {
                copy(out + r * dim);
            }
            ++r;
            return BSR_OK;
        }));
        *out_rows = r;
        return BSR_OK;
    })());
}

int bsr_vstore_get(const bsr_vstore* vs, uint64_t index, float* out, uint32_t capacity, uint32_t* out_len) {
    VS_GUARD(([&]() -> int {
        if (!vs || !out_len) return set_error(BSR_E_INVALID, "null argument");
        // get(index) = get_many(SliceArgs { offset: index as i32, length: 1 }).get(0)
        const int64_t off = (int64_t)(int32_t)(uint32_t)index;
        uint64_t start, stop;
        slice_bounds(off, 1, vs->count(), &start, &stop);
        bool found = false;
        VS_TRY(walk_rows(vs, start, stop, [&](uint32_t n, auto&& copy) -> int {
            if (found) return BSR_OK;
            if (out && n > capacity) return set_error(BSR_E_INVALID, "output too small (%u floats)", n);
            if (out) copy(out);
            *out_len = n;
            found = true;
            return BSR_OK;
        }));
        if (!found) return set_error(BSR_E_INVALID, "Index not found");
        return BSR_OK;
    })());
}

int bsr_vstore_append_many(bsr_vstore* vs, const float* rows, uint64_t n_rows, uint32_t dim) {
    VS_GUARD(([&]() -> int {
        if (!vs || (n_rows && !rows)) return set_error(BSR_E_INVALID, "null argument");
        vs->app_vals.insert(vs->app_vals.end(), rows, rows + n_rows * (uint64_t)dim);
        for (uint64_t i = 0; i < n_rows; ++i) vs->app_off.push_back(vs->app_off.back() + dim);
        return BSR_OK;
    })());
}

int bsr_vstore_persist(bsr_vstore* vs) {
    VS_GUARD(([&]() -> int {
        if (!vs) return set_error(BSR_E_INVALID, "null argument");
        std::error_code ec;
        const fs::path p(vs->path);
        if (p.has_parent_path() && !fs::exists(p.parent_path(), ec)) {
            fs::create_directories(p.parent_path(), ec);
            if (ec) return set_error(BSR_E_INVALID, "Failed to create directory: %s", ec.message().c_str());
        }
        // every row (null rows kept as nulls, so the height is unchanged), one List(Float32) column
        arrow::ListBuilder lb(arrow::default_memory_pool(), std::make_shared<arrow::FloatBuilder>(), list_type());
        auto* fb = static_cast<arrow::FloatBuilder*>(lb.value_builder());
        const uint64_t n = vs->count(), fr = vs->file_rows();
        uint64_t base = 0;
        if (vs->col) {
            for (const auto& chunk : vs->col->chunks()) {
                for (int64_t i = 0; i < chunk->length(); ++i) {
                    VS_TRY(visit_chunk_row(*chunk, i, [&](bool valid, const std::shared_ptr<arrow::Array>& values,
                                                          int64_t off, int64_t len) -> int {
                        if (!valid) {
                            auto st = lb.AppendNull();
                            return st.ok() ? BSR_OK : arrow_error(st, "append");
                        }
                        auto st = lb.Append();
                        if (!st.ok()) return arrow_error(st, "append");
                        const auto& fa = static_cast<const arrow::FloatArray&>(*values);
                        for (int64_t j = 0; j < len; ++j) {
                            st = fa.IsValid(off + j) ? fb->Append(fa.Value(off + j)) : fb->AppendNull();
                            if (!st.ok()) return arrow_error(st, "append");
                        }
                        return BSR_OK;
                    }));
                }
                base += (uint64_t)chunk->length();
            }
        }
        for (uint64_t g = fr; g < n; ++g) {
            auto st = lb.Append();
            if (!st.ok()) return arrow_error(st, "append");
            const uint64_t a = vs->app_off[g - fr], b = vs->app_off[g - fr + 1];
            st = fb->AppendValues(vs->app_vals.data() + a, (int64_t)(b - a));
            if (!st.ok()) return arrow_error(st, "append");
        }
        std::shared_ptr<arrow::Array> arr;
        auto st = lb.Finish(&arr);
        if (!st.ok()) return arrow_error(st, "finish");
        VS_TRY(write_table(vs->path, arr));
        if (!fs::exists(p, ec)) return set_error(BSR_E_INVALID, "File was not created: %s", vs->path.c_str());
        return BSR_OK;
    })());
}

int bsr_vstore_reload(bsr_vstore* vs, int force) {
    VS_GUARD(([&]() -> int {
        if (!vs) return set_error(BSR_E_INVALID, "null argument");
        std::shared_ptr<arrow::ChunkedArray> c;
        VS_TRY(read_parquet(vs->path, &c));
        if (c->length() == 0 && !force) return set_error(BSR_E_STATE, "Found a empty or invalid file");
        vs->col = c;
        vs->app_vals.clear();
        vs->app_off.assign(1, 0);
        return BSR_OK;
    })());
}

int bsr_vstore_reset(bsr_vstore* vs) {
    if (!vs) return set_error(BSR_E_INVALID, "null argument");
    vs->col.reset();
    vs->app_vals.clear();
    vs->app_off.assign(1, 0);
    return BSR_OK;
}

static int join_path(const char* dir, const std::string& name, char* out, size_t cap) {
    if (!dir || !out) return set_error(BSR_E_INVALID, "null argument");
    const std::string s = (fs::path(dir) / name).string();
    if (s.size() + 1 > cap) return set_error(BSR_E_INVALID, "path buffer too small (%zu bytes needed)", s.size() + 1);
    memcpy(out, s.c_str(), s.size() + 1);
    return BSR_OK;
}

int bsr_vstore_global_path(const char* dir, char* out, size_t cap) {
    VS_GUARD(join_path(dir, "global.parquet", out, cap));
}

int bsr_vstore_local_path(const char* dir, int32_t rank, char* out, size_t cap) {
    VS_GUARD(join_path(dir, "rank_" + std::to_string(rank) + ".parquet", out, cap));
}

int bsr_index_load_vstore(bsr_index* ix, const bsr_vstore* vs, int32_t rank, int32_t size) {
    VS_GUARD(([&]() -> int {
        if (!ix || !vs) return set_error(BSR_E_INVALID, "null argument");
        bsr_rank_interval iv;
        VS_TRY(bsr_interval_by_rank(rank, size, vs->count(), &iv));
        uint32_t dim = 0;
        VS_TRY(bsr_index_dim(ix, &dim));
        if (iv.start_index >= iv.end_index) return bsr_index_load(ix, nullptr, 0, iv.start_index);
        // stream the block in pieces of <= 1M rows (host staging stays bounded)
        constexpr uint64_t kPiece = 1u << 20;
        std::vector<float> buf;
        bool first = true;
        for (uint64_t s = iv.start_index; s < iv.end_index; s += kPiece) {
            const uint64_t len = std::min(kPiece, iv.end_index - s);
            buf.resize(len * dim);
            uint64_t got = 0;
            VS_TRY(bsr_vstore_read_slab(vs, (int64_t)s, len, dim, buf.data(), len, &got));
            if (first) VS_TRY(bsr_index_load(ix, buf.data(), got, iv.start_index));
            else if (got) VS_TRY(bsr_index_append(ix, buf.data(), got));
            first = false;
        }
        return BSR_OK;
    })());
}

}  // extern "C"
