// mops_netcdf.cpp -- netCDF classic-format (CDF-1/2/5) reader (include/mops_netcdf.h).
// Format: the published netCDF classic/64-bit-offset/64-bit-data file format
// specification (big-endian header + data, record variables interleaved per
// record).  Only what MPASOReader needs: dimensions, variable shapes, and
// whole-variable / single-record reads with type conversion.
#include "mops_netcdf.h"

#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

extern "C" __attribute__((visibility("hidden"))) mops_status mops_io_fail(mops_status st, const char* msg);

struct mops_nc {
    struct Var {
        std::string name;
        std::vector<int64_t> dimids;
        int32_t type = 0;
        int64_t begin = 0;
        bool record = false;
        int64_t rec_elems = 1;  // elements per record (record vars) or total (others)
    };
    std::string path;
    int version = 0;
    int64_t numrecs = 0;
    int64_t recsize = 0;
    int64_t record_dim = -1;
    std::vector<std::pair<std::string, int64_t>> dims;
    std::vector<Var> vars;
    std::map<std::string, size_t> var_index;
};

namespace {

int type_size(int32_t t) {
    switch (t) {
        case MOPS_NC_BYTE: case MOPS_NC_CHAR: case MOPS_NC_UBYTE: return 1;
        case MOPS_NC_SHORT: case MOPS_NC_USHORT: return 2;
        case MOPS_NC_INT: case MOPS_NC_FLOAT: case MOPS_NC_UINT: return 4;
        case MOPS_NC_DOUBLE: case MOPS_NC_INT64: case MOPS_NC_UINT64: return 8;
        default: return 0;
    }
}

struct Reader {
    FILE* f;
    bool ok = true;
    uint64_t be(int n) {
        unsigned char b[8];
        if (fread(b, 1, (size_t)n, f) != (size_t)n) { ok = false; return 0; }
        uint64_t v = 0;
        for (int i = 0; i < n; ++i) v = (v << 8) | b[i];
        return v;
    }
    int64_t i32() { return (int32_t)(uint32_t)be(4); }
    void skip(int64_t n) { if (n > 0 && fseeko(f, (off_t)n, SEEK_CUR) != 0) ok = false; }
    std::string name(int w) {
        const int64_t len = (int64_t)be(w);
        if (!ok || len < 0 || len > (1 << 20)) { ok = false; return {}; }
        std::string s((size_t)len, '\0');
        if (len && fread(&s[0], 1, (size_t)len, f) != (size_t)len) ok = false;
        skip((4 - len % 4) % 4);
        return s;
    }
};

const mops_nc::Var* find(const mops_nc* nc, const char* name) {
    auto it = nc->var_index.find(name ? name : "");
    return it == nc->var_index.end() ? nullptr : &nc->vars[it->second];
}

// Read `count` elements of `v` (record `record`) as raw big-endian bytes.
mops_status read_raw(const mops_nc* nc, const mops_nc::Var* v, int64_t record, int64_t count,
                     std::vector<unsigned char>& buf) {
    if (v->record) {
        if (record < 0 || record >= nc->numrecs) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read: record out of range");
    } else if (record != 0) {
        return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read: record given for a non-record variable");
    }
    if (count != v->rec_elems) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read: count does not match the variable");
    const int ts = type_size(v->type);
    const int64_t off = v->begin + (v->record ? record * nc->recsize : 0);
    FILE* f = fopen(nc->path.c_str(), "rb");
    if (!f) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read: cannot open file");
    buf.resize((size_t)(count * ts));
    bool ok = fseeko(f, (off_t)off, SEEK_SET) == 0 && fread(buf.data(), 1, buf.size(), f) == buf.size();
    fclose(f);
    if (!ok) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read: short read (truncated file?)");
    return MOPS_OK;
}

template <class T>
void convert(const std::vector<unsigned char>& b, int32_t type, int64_t n, T* out) {
    const unsigned char* p = b.data();
    for (int64_t i = 0; i < n; ++i) {
        switch (type) {
            case MOPS_NC_BYTE: out[i] = (T)(int8_t)p[i]; break;
            case MOPS_NC_UBYTE: case MOPS_NC_CHAR: out[i] = (T)p[i]; break;
            case MOPS_NC_SHORT: out[i] = (T)(int16_t)(uint16_t)((p[2 * i] << 8) | p[2 * i + 1]); break;
            case MOPS_NC_USHORT: out[i] = (T)(uint16_t)((p[2 * i] << 8) | p[2 * i + 1]); break;
            case MOPS_NC_INT: case MOPS_NC_UINT: case MOPS_NC_FLOAT: {
                uint32_t u = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) |
                             (uint32_t)p[4 * i + 3];
                if (type == MOPS_NC_INT) out[i] = (T)(int32_t)u;
                else if (type == MOPS_NC_UINT) out[i] = (T)u;
                else { float fl; std::memcpy(&fl, &u, 4); out[i] = (T)fl; }
                break;
            }
            default: {  // 8-byte types
                uint64_t u = 0;
                for (int k = 0; k < 8; ++k) u = (u << 8) | p[8 * i + k];
                if (type == MOPS_NC_DOUBLE) { double d; std::memcpy(&d, &u, 8); out[i] = (T)d; }
                else if (type == MOPS_NC_INT64) out[i] = (T)(int64_t)u;
                else out[i] = (T)u;
            }
        }
    }
}

}  // namespace

extern "C" {

mops_status mops_nc_open(const char* path, mops_nc** out) {
    if (!path || !out) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_open: null argument");
    *out = nullptr;
    FILE* f = fopen(path, "rb");
    if (!f) return mops_io_fail(MOPS_ERR_INVALID, (std::string("mops_nc_open: cannot open ") + path).c_str());
    Reader r{f};
    unsigned char magic[4] = {0, 0, 0, 0};
    if (fread(magic, 1, 4, f) != 4) { fclose(f); return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_open: short file"); }
    if (magic[0] == 0x89 && magic[1] == 'H' && magic[2] == 'D' && magic[3] == 'F') {
        fclose(f);
        return mops_io_fail(MOPS_ERR_UNSUPPORTED, "mops_nc_open: netCDF-4/HDF5 file (convert with nccopy -k cdf5)");
    }
    if (magic[0] != 'C' || magic[1] != 'D' || magic[2] != 'F' || (magic[3] != 1 && magic[3] != 2 && magic[3] != 5)) {
        fclose(f);
        return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_open: not a netCDF classic file");
    }
    mops_nc* nc = new mops_nc();
    nc->path = path;
    nc->version = magic[3];
    const int W = nc->version == 5 ? 8 : 4;         // NON_NEG width
    const int OW = nc->version == 1 ? 4 : 8;        // OFFSET width
    const uint64_t nrec_raw = r.be(W);
    const bool streaming = (W == 4 && nrec_raw == 0xFFFFFFFFull) || (W == 8 && nrec_raw == ~0ull);
    nc->numrecs = streaming ? -1 : (int64_t)nrec_raw;
    auto list_header = [&](uint32_t want, int64_t& n) {
        const uint32_t tag = (uint32_t)r.be(4);
        n = (int64_t)r.be(W);
        if (tag != 0 && tag != want) r.ok = false;
        if (tag == 0 && n != 0) r.ok = false;
    };
    auto skip_atts = [&]() {
        int64_t na = 0;
        list_header(0x0C, na);
        for (int64_t a = 0; a < na && r.ok; ++a) {
            r.name(W);
            const int32_t t = (int32_t)r.be(4);
            const int64_t nv = (int64_t)r.be(W);
            const int64_t bytes = nv * type_size(t);
            if (type_size(t) == 0 || nv < 0) { r.ok = false; break; }
            r.skip(bytes + (4 - bytes % 4) % 4);
        }
    };
    int64_t nd = 0;
    list_header(0x0A, nd);
    for (int64_t d = 0; d < nd && r.ok; ++d) {
        std::string nm = r.name(W);
        const int64_t len = (int64_t)r.be(W);
        if (len == 0) nc->record_dim = d;
        nc->dims.emplace_back(nm, len);
    }
    skip_atts();
    int64_t nv = 0;
    list_header(0x0B, nv);
    for (int64_t v = 0; v < nv && r.ok; ++v) {
        mops_nc::Var var;
        var.name = r.name(W);
        const int64_t rank = (int64_t)r.be(W);
        if (rank < 0 || rank > 64) { r.ok = false; break; }
        for (int64_t k = 0; k < rank; ++k) var.dimids.push_back((int64_t)r.be(W));
        skip_atts();
        var.type = (int32_t)r.be(4);
        r.be(W);  // vsize (recomputed: it saturates for > 4 GiB variables)
        var.begin = (int64_t)r.be(OW);
        for (size_t k = 0; k < var.dimids.size(); ++k) {
            const int64_t id = var.dimids[k];
            if (id < 0 || id >= (int64_t)nc->dims.size()) { r.ok = false; break; }
            if (id == nc->record_dim) {
                if (k != 0) r.ok = false;  // only the first dimension may be unlimited
                var.record = true;
            } else {
                var.rec_elems *= nc->dims[(size_t)id].second;
            }
        }
        if (type_size(var.type) == 0) r.ok = false;
        nc->var_index[var.name] = nc->vars.size();
        nc->vars.push_back(var);
    }
    if (!r.ok) {
        fclose(f);
        delete nc;
        return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_open: malformed netCDF header");
    }
    // one record = every record variable's slab, each padded to 4 bytes --
    // except a lone record variable, which is not padded
    int n_rec_vars = 0;
    int64_t first_begin = -1;
    for (auto& v : nc->vars)
        if (v.record) {
            const int64_t b = v.rec_elems * type_size(v.type);
            nc->recsize += b + (4 - b % 4) % 4;
            ++n_rec_vars;
            if (first_begin < 0 || v.begin < first_begin) first_begin = v.begin;
        }
    if (n_rec_vars == 1)
        for (auto& v : nc->vars)
            if (v.record) nc->recsize = v.rec_elems * type_size(v.type);
    if (nc->numrecs < 0) {  // streaming header: derive from the file size
        fseeko(f, 0, SEEK_END);
        const int64_t size = (int64_t)ftello(f);
        nc->numrecs = (nc->recsize > 0 && first_begin >= 0) ? (size - first_begin) / nc->recsize : 0;
    }
    if (nc->record_dim >= 0) nc->dims[(size_t)nc->record_dim].second = nc->numrecs;
    fclose(f);
    *out = nc;
    return MOPS_OK;
}

void mops_nc_close(mops_nc* nc) { delete nc; }

mops_status mops_nc_dim_len(const mops_nc* nc, const char* name, int64_t* len) {
    if (!nc || !name || !len) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_dim_len: null argument");
    for (auto& d : nc->dims)
        if (d.first == name) { *len = d.second; return MOPS_OK; }
    return mops_io_fail(MOPS_ERR_INVALID, (std::string("mops_nc_dim_len: no dimension ") + name).c_str());
}

mops_status mops_nc_var_info(const mops_nc* nc, const char* name, int32_t* type, int32_t* ndims, int64_t* shape,
                             int32_t* is_record) {
    if (!nc) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_var_info: null argument");
    const mops_nc::Var* v = find(nc, name);
    if (!v) return mops_io_fail(MOPS_ERR_INVALID, (std::string("mops_nc_var_info: no variable ") + (name ? name : "")).c_str());
    if (type) *type = v->type;
    if (ndims) *ndims = (int32_t)v->dimids.size();
    if (shape)
        for (size_t k = 0; k < v->dimids.size() && k < 8; ++k) shape[k] = nc->dims[(size_t)v->dimids[k]].second;
    if (is_record) *is_record = v->record ? 1 : 0;
    return MOPS_OK;
}

mops_status mops_nc_read_f64(const mops_nc* nc, const char* name, int64_t record, double* out, int64_t count) {
    const mops_nc::Var* v = nc ? find(nc, name) : nullptr;
    if (!v || !out) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read_f64: no such variable / null output");
    if (v->type == MOPS_NC_CHAR) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read_f64: NC_CHAR variable");
    std::vector<unsigned char> buf;
    mops_status st = read_raw(nc, v, record, count, buf);
    if (st != MOPS_OK) return st;
    convert<double>(buf, v->type, count, out);
    return MOPS_OK;
}

mops_status mops_nc_read_i64(const mops_nc* nc, const char* name, int64_t record, int64_t* out, int64_t count) {
    const mops_nc::Var* v = nc ? find(nc, name) : nullptr;
    if (!v || !out) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read_i64: no such variable / null output");
    if (v->type == MOPS_NC_FLOAT || v->type == MOPS_NC_DOUBLE || v->type == MOPS_NC_CHAR)
        return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read_i64: not an integer variable");
    std::vector<unsigned char> buf;
    mops_status st = read_raw(nc, v, record, count, buf);
    if (st != MOPS_OK) return st;
    convert<int64_t>(buf, v->type, count, out);
    return MOPS_OK;
}

mops_status mops_nc_read_bytes(const mops_nc* nc, const char* name, int64_t record, char* out, int64_t count) {
    const mops_nc::Var* v = nc ? find(nc, name) : nullptr;
    if (!v || !out) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read_bytes: no such variable / null output");
    if (type_size(v->type) != 1) return mops_io_fail(MOPS_ERR_INVALID, "mops_nc_read_bytes: not a byte/char variable");
    std::vector<unsigned char> buf;
    mops_status st = read_raw(nc, v, record, count, buf);
    if (st != MOPS_OK) return st;
    std::memcpy(out, buf.data(), (size_t)count);
    return MOPS_OK;
}

}  // extern "C"
