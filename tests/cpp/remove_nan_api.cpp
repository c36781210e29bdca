// remove_nan_api.cpp -- drives MOPS::RemoveNaNTrajectoriesAndReindex (include/mops/MOPS.h,
// the reference's src/Common/TrajectoryCommon.h:57-129) on a batch of ragged lines written by
// tests/test_remove_nan_gpu.py, the way test/test_trajector.cpp:26-194 drives it, and writes
// the cleaned lines back.
//
//   remove_nan_api <in.bin> <out.bin>
//
// in.bin : int64 n; per line: int64 lineID, int64 P, int64 V (velocity entries, <= P),
//          P x {x,y,z} f64, V x {vx,vy,vz} f64, P x t f64, P x s f64
// out.bin: int64 m; per kept line: int64 lineID, int64 P, P x {x,y,z,vx,vy,vz,t,s} f64, {last xyz} f64
#include <cstdint>
#include <fstream>
#include <iostream>
#include <vector>

#include "mops/MOPS.h"

template <class T>
static T get(std::ifstream& f) {
    T v{};
    f.read(reinterpret_cast<char*>(&v), sizeof(T));
    return v;
}

template <class T>
static void put(std::ofstream& f, T v) {
    f.write(reinterpret_cast<const char*>(&v), sizeof(T));
}

int main(int argc, char** argv) {
    if (argc != 3) {
        std::cerr << "usage: remove_nan_api <in.bin> <out.bin>\n";
        return 2;
    }
    std::ifstream in(argv[1], std::ios::binary);
    const int64_t n = get<int64_t>(in);
    std::vector<MOPS::TrajectoryLine> lines((size_t)n);
    for (auto& l : lines) {
        l.lineID = (int)get<int64_t>(in);
        const int64_t P = get<int64_t>(in), V = get<int64_t>(in);
        l.points.resize((size_t)P);
        l.velocity.resize((size_t)V);
        l.temperature.resize((size_t)P);
        l.salinity.resize((size_t)P);
        for (auto& p : l.points) p = {get<double>(in), get<double>(in), get<double>(in)};
        for (auto& v : l.velocity) v = {get<double>(in), get<double>(in), get<double>(in)};
        for (auto& t : l.temperature) t = get<double>(in);
        for (auto& s : l.salinity) s = get<double>(in);
    }
    if (!in) {
        std::cerr << "cannot read " << argv[1] << "\n";
        return 2;
    }
    std::vector<MOPS::TrajectoryLine> out;
    try {
        out = MOPS::RemoveNaNTrajectoriesAndReindex(lines);
    } catch (const std::exception& e) {
        std::cerr << e.what() << "\n";
        return 1;
    }
    std::ofstream o(argv[2], std::ios::binary);
    put<int64_t>(o, (int64_t)out.size());
    for (const auto& l : out) {
        put<int64_t>(o, l.lineID);
        put<int64_t>(o, (int64_t)l.points.size());
        for (size_t j = 0; j < l.points.size(); ++j) {
            put(o, l.points[j].x); put(o, l.points[j].y); put(o, l.points[j].z);
            put(o, l.velocity[j].x); put(o, l.velocity[j].y); put(o, l.velocity[j].z);
            put(o, l.temperature[j]); put(o, l.salinity[j]);
        }
        put(o, l.lastPoint.x); put(o, l.lastPoint.y); put(o, l.lastPoint.z);
    }
    return o ? 0 : 1;
}
