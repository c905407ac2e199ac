// Qt raster micro-golden generator (build container only; see tools/make_raster_goldens.py).
//
// The reference rasterises every observation with Qt5's raster QPainter into a
// 64x64 32-bit QImage (upstream contract: procgen/src/game.cpp:8-23 bgr32_to_rgb888,
// Game::render_to_buf; the fork's browser-canvas shim is not reproducible, see
// SURVEY.md section 0).  This program replays painter command lists through the
// REAL Qt 5.9.7 raster engine present in this image so the oracle's restatement
// of those semantics (oracle/procgen_oracle.c, qt_* functions) can be pinned
// bit-for-bit against it.
//
// stdin (little endian):  u32 ncases; per case: u32 canvas_fmt (4 = RGB32),
//   u32 canvas[64*64], u32 ncmds; per cmd:
//     u32 kind  (0 drawImage(QRectF, QImage) ; 1 fillRect(QRectF, QColor) ; 2 fillRect(QRect, QColor))
//     f64 x, y, w, h ; f64 opacity ; u32 mirrored ; u32 rotate_deg_x1000 (signed, 0 = none)
//     kind 0: u32 img_fmt (6 = ARGB32_Premultiplied, 4 = RGB32), u32 w, u32 h, u32 pixels[w*h]
//     kind 1/2: u32 color (0xAARRGGBB)
//     kind 3: f64 deg, then as kind 0: drawImage(QRectF(-w/2, -h/2, w, h)) after
//             translate(x + w/2, y + h/2) and rotate(deg) (basic-abstract-game.cpp:908-916)
// stdout: per case u32 canvas[64*64] after painting.
#include <QImage>
#include <QPainter>
#include <cstdint>
#include <cstdio>
#include <vector>

template <typename T> static T rd() {
    T v;
    if (fread(&v, sizeof(T), 1, stdin) != 1) { fprintf(stderr, "short read\n"); exit(3); }
    return v;
}

int main() {
    uint32_t ncases = rd<uint32_t>();
    for (uint32_t c = 0; c < ncases; c++) {
        uint32_t cfmt = rd<uint32_t>();
        QImage canvas(64, 64, (QImage::Format)cfmt);
        for (int y = 0; y < 64; y++) {
            uint32_t *line = (uint32_t *)canvas.scanLine(y);
            for (int x = 0; x < 64; x++) line[x] = rd<uint32_t>();
        }
        uint32_t ncmds = rd<uint32_t>();
        {
            QPainter p(&canvas);
            for (uint32_t k = 0; k < ncmds; k++) {
                uint32_t kind = rd<uint32_t>();
                double x = rd<double>(), y = rd<double>(), w = rd<double>(), h = rd<double>();
                double opacity = rd<double>();
                uint32_t mirrored = rd<uint32_t>();
                int32_t rot = (int32_t)rd<uint32_t>();
                double deg = 0;
                if (kind == 3) deg = rd<double>();
                if (kind == 0 || kind == 3) {
                    uint32_t ifmt = rd<uint32_t>(), iw = rd<uint32_t>(), ih = rd<uint32_t>();
                    QImage img(iw, ih, (QImage::Format)ifmt);
                    for (uint32_t yy = 0; yy < ih; yy++) {
                        uint32_t *line = (uint32_t *)img.scanLine(yy);
                        for (uint32_t xx = 0; xx < iw; xx++) line[xx] = rd<uint32_t>();
                    }
                    QImage use = mirrored ? img.mirrored(true, false) : img;
                    bool st = opacity != 1.0;
                    if (st) { p.save(); p.setOpacity(opacity); }
                    if (kind == 3) {
                        p.save();
                        p.translate(x + w / 2, y + h / 2);
                        p.rotate(deg);
                        p.drawImage(QRectF(-w / 2, -h / 2, w, h), use);
                        p.restore();
                    } else if (rot == 0) {
                        p.drawImage(QRectF(x, y, w, h), use);
                    } else {
                        p.save();
                        p.translate(x + w / 2, y + h / 2);
                        p.rotate(rot / 1000.0);
                        p.drawImage(QRectF(-w / 2, -h / 2, w, h), use);
                        p.restore();
                    }
                    if (st) p.restore();
                } else {
                    uint32_t col = rd<uint32_t>();
                    QColor qc = QColor::fromRgba(col);
                    if (kind == 1) p.fillRect(QRectF(x, y, w, h), qc);
                    else p.fillRect(QRect((int)x, (int)y, (int)w, (int)h), qc);
                }
            }
        }
        for (int y = 0; y < 64; y++) fwrite(canvas.constScanLine(y), 4, 64, stdout);
    }
    return 0;
}
