// Asset decoder used ONLY to build the committed asset pack (tools/make_asset_pack.py).
//
// It reproduces the reference's loading contract exactly by calling the same
// third-party library the reference uses (Qt5 QImage, present in this image at
// /opt/conda, Qt 5.9.7):
//   sprites:      QImage(path).convertToFormat(QImage::Format_ARGB32_Premultiplied)
//   backgrounds:  QImage(path).convertToFormat(QImage::Format_RGB32)
// (reference: procgen/src/resources.cpp:20-30 load_resource_ptr, :964 (RGB32
// backgrounds), :969 (ARGB32_Premultiplied sprites)).
//
// Input on stdin: lines "<kind> <root-relative path>", kind = S (sprite) or B (background).
// Output (argv[2]): for every line, u32 kind, u32 w, u32 h, then w*h u32 pixels (0xAARRGGBB).
#include <QImage>
#include <cstdio>
#include <cstdint>
#include <iostream>
#include <string>

int main(int argc, char **argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s <asset_root/> <out.bin> < list\n", argv[0]);
        return 2;
    }
    std::string root = argv[1];
    FILE *out = fopen(argv[2], "wb");
    if (!out) return 2;
    std::string kind, rel;
    while (std::cin >> kind >> rel) {
        QImage raw(QString::fromStdString(root + rel));
        uint32_t k = kind == "B" ? 1u : 0u;
        if (raw.isNull()) {
            // missing file (e.g. misc_assets/mud.png): record a 0x0 image
            uint32_t hdr[3] = {k, 0u, 0u};
            fwrite(hdr, 4, 3, out);
            fprintf(stderr, "missing %s\n", rel.c_str());
            continue;
        }
        QImage img = raw.convertToFormat(k ? QImage::Format_RGB32 : QImage::Format_ARGB32_Premultiplied);
        uint32_t hdr[3] = {k, (uint32_t)img.width(), (uint32_t)img.height()};
        fwrite(hdr, 4, 3, out);
        for (int y = 0; y < img.height(); y++) {
            fwrite(img.constScanLine(y), 4, img.width(), out);
        }
    }
    fclose(out);
    return 0;
}
