// The C++ wrapper's frame output without a GPU: Screen::writeBitmapToFile and saveFeaturesRecord
// (render.cpp:281-287), as a reference-side caller would use them.  argv: <out.bmp> <record dir>
#include <romis_amd/restir.hpp>

#include <cstdio>

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    romis::Screen screen(5, 3);
    for (int y = 0; y < 3; y++)
        for (int x = 0; x < 5; x++) {
            float* p = screen.pixel(x, y);
            p[0] = 0.1f * x - 0.05f; p[1] = 0.4f * y; p[2] = 1.2f - 0.2f * x;
        }
    screen.writeBitmapToFile(argv[1]);
    romis::Features f;
    f.gamma = 2.2f;
    f.num_samples_in_reservoir = 4;
    const std::filesystem::path rec = romis::saveFeaturesRecord(f, argv[2]);
    std::printf("%s\n", rec.string().c_str());
    return 0;
}
