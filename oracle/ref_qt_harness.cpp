// Driver for the AssetGen pins (TEST INFRASTRUCTURE ONLY).
//
// Compiled by `make -C oracle ref` together with the reference's own, unmodified
// /root/reference/procgen/src/assetgen.cpp and randgen.cpp, read in place, against the REAL Qt
// 5.9.7 of this image (/opt/conda) -- assetgen.h includes only randgen.h and Qt headers, so this
// part of the reference builds from its own files with no stand-in.  Output only to oracle/_ref/
// (git-ignored).  The oracle's restatement (procgen_oracle.c ag_*) and the device painter are
// checked against these functions (tests/test_assetgen_pins.py).
#include <QColor>
#include <QImage>
#include <QPainter>
#include <QPainterPath>
#include <cstdint>
#include <cstring>
#include <memory>

#include "assetgen.h"
#include "qt-utils.h"
#include "randgen.h"

static void copy_out(const QImage &img, uint32_t *out) {
    for (int y = 0; y < img.height(); y++)
        memcpy(out + (size_t)y * img.width(), img.constScanLine(y), (size_t)img.width() * 4);
}

extern "C" {

// AssetGen::generate_resource on a w x h image of `fmt` (4 = RGB32: backgrounds,
// basic-abstract-game.cpp:60-63, 778-782; 5 = ARGB32: generated sprites, :101-107) with a RandGen
// seeded `seed` and then advanced by `pre_draws` randint() calls (the reset draws before it);
// `init` fills the image first (the reference paints over whatever the QImage holds).  Writes the
// w*h pixels; returns the generator's next randint() after painting (pins how many it consumed).
int32_t ref_generate_resource(int32_t seed, int pre_draws, int w, int h, int fmt, int num_recurse, int blotch_scale,
                              int is_rect, uint32_t init, uint32_t *out) {
    RandGen rg;
    rg.seed(seed);
    for (int i = 0; i < pre_draws; i++) rg.randint();
    auto img = std::make_shared<QImage>(w, h, (QImage::Format)fmt);
    img->fill(init);
    AssetGen gen(&rg);
    gen.generate_resource(img, num_recurse, blotch_scale, is_rect != 0);
    copy_out(*img, out);
    return rg.randint();
}

// One Qt primitive on a w x h canvas of `fmt` (initial pixels `inout`), the way AssetGen calls it:
// kind 0 fillRect(QRectF, QColor(argb)); kind 1 setBrush(QBrush(c1)) + setPen(QPen(c2)) +
// drawEllipse(QRectF); kind 2 as 1 with the brush only (Qt::NoPen); kind 3 as 1 with the pen only
// (Qt::NoBrush).  `source` selects CompositionMode_Source (paint_shape_resource) over SourceOver.
void ref_qt_shape(int w, int h, int fmt, int kind, double x, double y, double rw, double rh, uint32_t c1,
                  uint32_t c2, int source, uint32_t *inout) {
    QImage img(w, h, (QImage::Format)fmt);
    for (int r = 0; r < h; r++) memcpy(img.scanLine(r), inout + (size_t)r * w, (size_t)w * 4);
    {
        QPainter p(&img);
        if (source) p.setCompositionMode(QPainter::CompositionMode_Source);
        QRectF rect(x, y, rw, rh);
        if (kind == 0) {
            p.fillRect(rect, QColor::fromRgba(c1));
        } else {
            if (kind == 3) p.setBrush(Qt::NoBrush);
            else p.setBrush(QBrush(QColor::fromRgba(c1)));
            if (kind == 2) p.setPen(Qt::NoPen);
            else p.setPen(QPen(QColor::fromRgba(c2)));
            p.drawEllipse(rect);
        }
    }
    copy_out(img, inout);
}

// A polyline (pts = x0, y0, x1, y1, ...; n points) stroked with QPen(color) (width 1: the cosmetic
// stroker's line path), for probing the stroker segment by segment.
void ref_qt_polyline(int w, int h, const double *pts, int n, uint32_t color, uint32_t *inout) {
    QImage img(w, h, QImage::Format_RGB32);
    for (int r = 0; r < h; r++) memcpy(img.scanLine(r), inout + (size_t)r * w, (size_t)w * 4);
    {
        QPainter p(&img);
        QPainterPath path;
        path.moveTo(pts[0], pts[1]);
        for (int i = 1; i < n; i++) path.lineTo(pts[2 * i], pts[2 * i + 1]);
        p.setBrush(Qt::NoBrush);
        p.setPen(QPen(QColor::fromRgba(color)));
        p.drawPath(path);
    }
    copy_out(img, inout);
}

// drawImage(QRectF(x, y, w, h), img) of an iw x ih image of `fmt` (optionally mirrored first, as the
// reference's reflections) onto a 64x64 RGB32 canvas `inout`: how generated ARGB32 sprites are drawn
void ref_qt_draw_image(const uint32_t *img, int iw, int ih, int fmt, int mirrored, double x, double y, double w,
                       double h, uint32_t *inout) {
    QImage src(iw, ih, (QImage::Format)fmt);
    for (int r = 0; r < ih; r++) memcpy(src.scanLine(r), img + (size_t)r * iw, (size_t)iw * 4);
    QImage canvas(64, 64, QImage::Format_RGB32);
    for (int r = 0; r < 64; r++) memcpy(canvas.scanLine(r), inout + (size_t)r * 64, 64 * 4);
    {
        QPainter p(&canvas);
        p.drawImage(QRectF(x, y, w, h), mirrored ? src.mirrored(true, false) : src);
    }
    copy_out(canvas, inout);
}

// QImage::mirrored(true, false) of a w x h image (basic-abstract-game.cpp:121-122)
void ref_qt_mirrored(int w, int h, int fmt, const uint32_t *in, uint32_t *out) {
    QImage img(w, h, (QImage::Format)fmt);
    for (int r = 0; r < h; r++) memcpy(img.scanLine(r), in + (size_t)r * w, (size_t)w * 4);
    copy_out(img.mirrored(true, false), out);
}

// qt-utils.h:12-19 adjust_rect over (x, y, w, h) quadruples (QRectF arithmetic in qreal = double)
void ref_adjust_rect(const double *base, const double *adj, double *out, int64_t n) {
    for (int64_t i = 0; i < n; i++) {
        QRectF r = adjust_rect(QRectF(base[4 * i], base[4 * i + 1], base[4 * i + 2], base[4 * i + 3]),
                               QRectF(adj[4 * i], adj[4 * i + 1], adj[4 * i + 2], adj[4 * i + 3]));
        out[4 * i] = r.x(); out[4 * i + 1] = r.y(); out[4 * i + 2] = r.width(); out[4 * i + 3] = r.height();
    }
}

// qt-utils.h:21-28 to_shade
void ref_to_shade(const float *f, int32_t *out, int64_t n) {
    for (int64_t i = 0; i < n; i++) out[i] = to_shade(f[i]);
}

} // extern "C"
