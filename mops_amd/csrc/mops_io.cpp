// mops_io.cpp -- host writers for the trajectory output formats (include/mops_io.h).
// They stream already-converted lines (mops_lines_geo runs on the GPU) to disk.
#include "mops_io.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <string>
#include <vector>

extern "C" __attribute__((visibility("hidden"))) mops_status mops_io_fail(mops_status st, const char* msg);  // mops_engine.hip

namespace {

std::string with_ext(const std::string& f, const std::string& ext) {  // checkAndModifyExtension (:305-312)
    if (f.size() >= ext.size() && f.compare(f.size() - ext.size(), ext.size(), ext) == 0) return f;
    return f + "." + ext;
}

// pathlib.Path.with_suffix('.meta.json')
std::string meta_path(const std::string& p) {
    const size_t slash = p.find_last_of('/');
    const size_t dot = p.find_last_of('.');
    const size_t name0 = (slash == std::string::npos) ? 0 : slash + 1;
    if (dot != std::string::npos && dot > name0) return p.substr(0, dot) + ".meta.json";
    return p + ".meta.json";
}

template <class T>
void put(std::ofstream& f, T v) {
    f.write(reinterpret_cast<const char*>(&v), sizeof(T));
}

struct VtpData {
    std::vector<float> pts;        // vtkPoints default type is float
    std::vector<double> tmp, sal, vmag;
    std::vector<int64_t> conn, offs;
};

void ascii_array(std::ofstream& f, const char* type, const char* name, int comps, const void* data, size_t count,
                 bool is_float32, bool is_int) {
    f << "        <DataArray type=\"" << type << "\"";
    if (name) f << " Name=\"" << name << "\"";
    if (comps > 1) f << " NumberOfComponents=\"" << comps << "\"";
    f << " format=\"ascii\">\n";
    f.precision(17);
    for (size_t i = 0; i < count; ++i) {
        if (is_int) f << static_cast<const int64_t*>(data)[i];
        else if (is_float32) f << static_cast<const float*>(data)[i];
        else f << static_cast<const double*>(data)[i];
        f << ((i + 1) % 6 == 0 || i + 1 == count ? "\n" : " ");
    }
    f << "        </DataArray>\n";
}

}  // namespace

extern "C" {

mops_status mops_write_lines_vtp(const char* path, int64_t n, int64_t P, const double* h_geo,
                                 const double* h_temperature, const double* h_salinity, int binary) {
    if (!path || n < 0 || P < 0 || (n > 0 && P > 0 && !h_geo)) return mops_io_fail(MOPS_ERR_INVALID, "mops_write_lines_vtp: invalid argument");
    const double kNaN = std::numeric_limits<double>::quiet_NaN();
    const double earthRadius = 6371010.0;  // :360
    VtpData d;
    d.pts.reserve((size_t)(n * P * 3));
    int64_t line_start = 0;
    for (int64_t l = 0; l < n && P > 0; ++l) {
        bool first = true;
        double prev_lon = 0.0;
        int64_t cur = 0;  // points in the open polyline
        for (int64_t i = 0; i < P; ++i) {
            const double* g = h_geo + (l * P + i) * 4;
            const double lat = g[0], lon = g[1], r = g[2];
            if (!first && ((prev_lon < -170 && lon > 170) || (prev_lon > 170 && lon < -170))) {
                line_start += cur;  // close the polyline, start a new one
                d.offs.push_back(line_start);
                cur = 0;
            }
            const int64_t pid = (int64_t)(d.pts.size() / 3);
            d.pts.push_back((float)lon);
            d.pts.push_back((float)lat);
            d.pts.push_back((float)(earthRadius - r));
            d.conn.push_back(pid);
            ++cur;
            d.tmp.push_back(h_temperature ? h_temperature[l * P + i] : kNaN);
            d.sal.push_back(h_salinity ? h_salinity[l * P + i] : kNaN);
            d.vmag.push_back(g[3]);
            prev_lon = lon;
            first = false;
        }
        if (cur > 0) {
            line_start += cur;
            d.offs.push_back(line_start);
        }
    }
    const std::string fn = with_ext(path, "vtp");
    std::ofstream f(fn, std::ios::binary);
    if (!f) return mops_io_fail(MOPS_ERR_INVALID, ("cannot open " + fn).c_str());
    const size_t np = d.pts.size() / 3, nl = d.offs.size();
    f << "<?xml version=\"1.0\"?>\n"
      << "<VTKFile type=\"PolyData\" version=\"1.0\" byte_order=\"LittleEndian\" header_type=\"UInt64\">\n"
      << "  <PolyData>\n"
      << "    <Piece NumberOfPoints=\"" << np << "\" NumberOfVerts=\"0\" NumberOfLines=\"" << nl
      << "\" NumberOfStrips=\"0\" NumberOfPolys=\"0\">\n";
    if (!binary) {
        f << "      <PointData>\n";
        ascii_array(f, "Float64", "temperature", 1, d.tmp.data(), d.tmp.size(), false, false);
        ascii_array(f, "Float64", "salinity", 1, d.sal.data(), d.sal.size(), false, false);
        ascii_array(f, "Float64", "velocity_mag", 1, d.vmag.data(), d.vmag.size(), false, false);
        f << "      </PointData>\n      <Points>\n";
        ascii_array(f, "Float32", "Points", 3, d.pts.data(), d.pts.size(), true, false);
        f << "      </Points>\n      <Lines>\n";
        ascii_array(f, "Int64", "connectivity", 1, d.conn.data(), d.conn.size(), false, true);
        ascii_array(f, "Int64", "offsets", 1, d.offs.data(), d.offs.size(), false, true);
        f << "      </Lines>\n    </Piece>\n  </PolyData>\n</VTKFile>\n";
    } else {
        struct Arr { const char* type; const char* name; int comps; const void* data; uint64_t bytes; };
        const Arr arrs[] = {
            {"Float64", "temperature", 1, d.tmp.data(), d.tmp.size() * 8},
            {"Float64", "salinity", 1, d.sal.data(), d.sal.size() * 8},
            {"Float64", "velocity_mag", 1, d.vmag.data(), d.vmag.size() * 8},
            {"Float32", "Points", 3, d.pts.data(), d.pts.size() * 4},
            {"Int64", "connectivity", 1, d.conn.data(), d.conn.size() * 8},
            {"Int64", "offsets", 1, d.offs.data(), d.offs.size() * 8},
        };
        uint64_t off[6], acc = 0;
        for (int i = 0; i < 6; ++i) { off[i] = acc; acc += 8 + arrs[i].bytes; }
        auto tag = [&](int i) {
            f << "        <DataArray type=\"" << arrs[i].type << "\" Name=\"" << arrs[i].name << "\"";
            if (arrs[i].comps > 1) f << " NumberOfComponents=\"" << arrs[i].comps << "\"";
            f << " format=\"appended\" offset=\"" << off[i] << "\"/>\n";
        };
        f << "      <PointData>\n"; tag(0); tag(1); tag(2); f << "      </PointData>\n";
        f << "      <Points>\n"; tag(3); f << "      </Points>\n";
        f << "      <Lines>\n"; tag(4); tag(5); f << "      </Lines>\n";
        f << "    </Piece>\n  </PolyData>\n  <AppendedData encoding=\"raw\">\n   _";
        for (int i = 0; i < 6; ++i) {
            put<uint64_t>(f, arrs[i].bytes);
            f.write(static_cast<const char*>(arrs[i].data), (std::streamsize)arrs[i].bytes);
        }
        f << "\n  </AppendedData>\n</VTKFile>\n";
    }
    if (!f) return mops_io_fail(MOPS_ERR_INVALID, ("write failed: " + fn).c_str());
    return MOPS_OK;
}

mops_status mops_write_lines_txt(const char* path, int64_t n, int64_t P, const double* h_points,
                                 const double* h_velocity) {
    if (!path || n < 0 || P < 0 || (n > 0 && P > 0 && (!h_points || !h_velocity)))
        return mops_io_fail(MOPS_ERR_INVALID, "mops_write_lines_txt: invalid argument");
    std::ofstream outFile(path);
    if (!outFile.is_open()) return mops_io_fail(MOPS_ERR_INVALID, "mops_write_lines_txt: cannot open file");
    outFile << "Line_Index Point_Index Position_X Position_Y Position_Z Velocity_X Velocity_Y Velocity_Z\n";
    for (int64_t l = 0; l < n; ++l)
        for (int64_t i = 0; i < P; ++i) {
            const double* p = h_points + (l * P + i) * 3;
            const double* v = h_velocity + (l * P + i) * 3;
            outFile << l << " " << i << " " << p[0] << " " << p[1] << " " << p[2] << " " << v[0] << " " << v[1]
                    << " " << v[2] << "\n";
        }
    if (!outFile) return mops_io_fail(MOPS_ERR_INVALID, "mops_write_lines_txt: write failed");
    return MOPS_OK;
}

mops_status mops_write_pathline_binary(const char* path, int64_t n, int64_t P, const double* h_geo,
                                       const double* h_velocity, const double* h_temperature,
                                       const double* h_salinity, int include_velocity, int include_scalars) {
    if (!path || n < 0 || n > INT32_MAX || P < 0 || P > INT32_MAX || (n > 0 && P > 0 && !h_geo))
        return mops_io_fail(MOPS_ERR_INVALID, "mops_write_pathline_binary: invalid argument");
    std::ofstream f(path, std::ios::binary);
    if (!f) return mops_io_fail(MOPS_ERR_INVALID, "mops_write_pathline_binary: cannot open file");
    std::vector<std::pair<int64_t, int64_t>> offsets;
    put<int32_t>(f, (int32_t)n);
    for (int64_t l = 0; l < n; ++l) {
        const int64_t start = (int64_t)f.tellp();
        put<int32_t>(f, (int32_t)P);
        for (int64_t i = 0; i < P; ++i) {
            const double* g = h_geo + (l * P + i) * 4;
            put<double>(f, g[0]);
            put<double>(f, g[1]);
            if (include_velocity) {
                if (h_velocity) {
                    const double* v = h_velocity + (l * P + i) * 3;
                    put<double>(f, v[0]); put<double>(f, v[1]); put<double>(f, g[3]);
                } else {
                    put<double>(f, 0.0); put<double>(f, 0.0); put<double>(f, 0.0);
                }
            }
            if (include_scalars) {
                put<double>(f, h_temperature ? h_temperature[l * P + i] : 0.0);
                put<double>(f, h_salinity ? h_salinity[l * P + i] : 0.0);
            }
        }
        offsets.emplace_back(start, P);
    }
    if (!f) return mops_io_fail(MOPS_ERR_INVALID, "mops_write_pathline_binary: write failed");
    std::ofstream m(meta_path(path));
    if (!m) return mops_io_fail(MOPS_ERR_INVALID, "mops_write_pathline_binary: cannot open meta file");
    m << "{\n  \"format_version\": \"1.0\",\n  \"num_particles\": " << n << ",\n  \"fields\": [\n    \"lat\",\n    \"lon\"";
    if (include_velocity) m << ",\n    \"velocity_u\",\n    \"velocity_v\",\n    \"speed\"";
    if (include_scalars) m << ",\n    \"temperature\",\n    \"salinity\"";
    m << "\n  ],\n  \"data_type\": \"float64\",\n  \"byte_order\": \"little\",\n  \"particle_offsets\": [";
    for (size_t i = 0; i < offsets.size(); ++i)
        m << (i ? "," : "") << "\n    {\n      \"start\": " << offsets[i].first << ",\n      \"points\": "
          << offsets[i].second << "\n    }";
    m << (offsets.empty() ? "]" : "\n  ]") << "\n}";
    return m ? MOPS_OK : mops_io_fail(MOPS_ERR_INVALID, "mops_write_pathline_binary: meta write failed");
}

}  // extern "C"
