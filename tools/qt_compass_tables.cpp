// Qt raster tables for jumper's compass overlay (build container only; see
// tools/make_compass_tables.py).
//
// jumper.cpp:137-177 (draw_compass) paints, after the foreground:
//   * the dial: drawEllipse(QRectF compass_rect) with pen = brush = QColor(168, 166, 158), pen width 1;
//   * the needle: drawLine(int, int, int, int) -- the float arguments select QPainter's int overload --
//     with a width-0 (cosmetic) pen of QColor(252, 186, 3): pen_thickness = 64 / (256 / compass_dim)
//     < 1 goes through set_pen_brush_color's `int thickness`;
//   * the distance bar: fillRect(QRectF) (restated in the oracle, pinned by qt_raster_fill_goldens);
//   * while double-jumping in the air: drawEllipse(QRect(...)) with NoPen and QColor(255, 255, 255, 120).
// Every colour is opaque except the last, and the geometry of the dial and of the needle's start
// only depends on (distribution mode, center_agent).  So the REAL Qt 5.9.7 raster engine of this
// image paints, for each configuration, the dial and the needle to every endpoint it can reach on
// an empty canvas; the changed pixels are the table the oracle and the engine stamp.  The jump
// ellipse is tabulated per QRect size (a translation-invariant integer-rect path, checked here)
// and its blend is checked against a random background.
//
// stdout (little-endian int32 / uint64):
//   per configuration cfg = hard(0/1) + 2 * uncentered(0/1):
//     i32 x1, y1 (needle start), i32 bx0, by0, bnx, bny (endpoint box), f32 cx, cy, cr,
//     u64 dial[64], u64 needle[bny][bnx][64]
//   jump ellipses: i32 maxw, maxh; u64 mask[maxw + 1][maxh + 1][64] for QRect(20, 20, w, h)
//   blend check: u32 bg[4096], u32 out[4096] for QRect(3, 4, 40, 30) over bg
#include <QImage>
#include <QPainter>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

static void put(const void *p, size_t n) { fwrite(p, 1, n, stdout); }
static void put_i(int32_t v) { put(&v, 4); }
static void put_f(float v) { put(&v, 4); }

static void mask_of(const QImage &img, uint64_t *rows) {
    for (int y = 0; y < 64; y++) {
        const uint32_t *line = (const uint32_t *)img.constScanLine(y);
        uint64_t m = 0;
        for (int x = 0; x < 64; x++)
            if (line[x] != 0) m |= 1ull << x;
        rows[y] = m;
    }
}

static QImage blank() {
    QImage img(64, 64, QImage::Format_ARGB32_Premultiplied);
    img.fill(0u);
    return img;
}

int main() {
    for (int cfg = 0; cfg < 4; cfg++) {
        const bool hard = cfg & 1, uncentered = cfg & 2;
        // jumper.cpp:212-232: visibility 12 / 16, compass_dim 3 / 2; world 20 / 40
        float visibility = hard ? 16 : 12;
        const float compass_dim = hard ? 2 : 3;
        const int main_width = hard ? 40 : 20;
        if (uncentered) visibility = main_width; // prepare_for_drawing (basic-abstract-game.cpp:832-838)
        const float raw_unit = 64 / visibility;  // :840-844 (rect_height 64)
        const float unit = raw_unit * (64 / 64.0);
        const float view_dim = 64.0 / raw_unit;
        // get_abs_rect(view_dim - compass_dim - .25, .25, compass_dim, compass_dim) (:812-814)
        const float ax = view_dim - compass_dim - .25, ay = .25;
        const QRectF compass_rect(ax * unit, ay * unit, compass_dim * unit, compass_dim * unit);
        const float cx = compass_rect.center().x();
        const float cy = compass_rect.center().y();
        const float cr = compass_rect.width() / 2 * .95;
        const int x1 = (int)cx, y1 = (int)cy;
        const int bx0 = (int)std::floor(cx - cr) - 1, by0 = (int)std::floor(cy - cr) - 1;
        const int bnx = (int)std::floor(cx + cr) + 2 - bx0, bny = (int)std::floor(cy + cr) + 2 - by0;
        put_i(x1); put_i(y1); put_i(bx0); put_i(by0); put_i(bnx); put_i(bny);
        put_f(cx); put_f(cy); put_f(cr);
        uint64_t rows[64];
        {
            QImage img = blank();
            QPainter p(&img);
            QColor clock_color(168, 166, 158);
            p.setBrush(QBrush(clock_color));
            p.setPen(QPen(clock_color, 1));
            p.drawEllipse(compass_rect);
            p.end();
            mask_of(img, rows);
            put(rows, sizeof(rows));
        }
        const float pen_thickness = 64 / (256.0 / compass_dim);
        for (int j = 0; j < bny; j++) {
            for (int i = 0; i < bnx; i++) {
                QImage img = blank();
                QPainter p(&img);
                QColor hl(252, 186, 3);
                p.setBrush(QBrush(hl));
                p.setPen(QPen(hl, (int)pen_thickness));
                p.drawLine(x1, y1, bx0 + i, by0 + j);
                p.end();
                mask_of(img, rows);
                put(rows, sizeof(rows));
            }
        }
    }
    const int maxw = 8, maxh = 4;
    put_i(maxw);
    put_i(maxh);
    for (int w = 0; w <= maxw; w++) {
        for (int h = 0; h <= maxh; h++) {
            uint64_t rows[64], rows2[64];
            for (int pass = 0; pass < 2; pass++) {
                const int ox = pass ? 31 : 20, oy = pass ? 13 : 20;
                QImage img = blank();
                QPainter p(&img);
                p.setBrush(QColor(255, 255, 255, 120));
                p.setPen(Qt::NoPen);
                p.drawEllipse(QRect(ox, oy, w, h));
                p.end();
                mask_of(img, pass ? rows2 : rows);
            }
            for (int y = 0; y < 64; y++) { // translation invariance: (31, 13) == (20, 20) + (11, -7)
                const uint64_t want = (y + 7 < 64) ? (rows[y + 7] << 11) : 0;
                if (rows2[y] != want) {
                    fprintf(stderr, "jump ellipse %dx%d is not translation invariant\n", w, h);
                    return 2;
                }
            }
            put(rows, sizeof(rows));
        }
    }
    {
        QImage img(64, 64, QImage::Format_RGB32);
        srand(7);
        for (int y = 0; y < 64; y++) {
            uint32_t *line = (uint32_t *)img.scanLine(y);
            for (int x = 0; x < 64; x++) line[x] = 0xff000000u | (uint32_t)((rand() & 0xffff) << 8 | (rand() & 0xff));
        }
        put(img.constBits(), 4096 * 4);
        QPainter p(&img);
        p.setBrush(QColor(255, 255, 255, 120));
        p.setPen(Qt::NoPen);
        p.drawEllipse(QRect(3, 4, 40, 30));
        p.end();
        put(img.constBits(), 4096 * 4);
    }
    return 0;
}
