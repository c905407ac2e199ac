// Probe of the real Qt 5.9.7 raster engine for render_mode="rgb_array" (build container only):
// the 512x512 frame is painted with Antialiasing + SmoothPixmapTransform (game.cpp:97-107).
// Built as a shared library (tools/Makefile-free: see tools/make_smooth_goldens.py) so the oracle's
// restatement of the smooth paths can be checked case by case and golden vectors generated.
#include <QImage>
#include <QPainter>
#include <cstdint>
#include <cstring>

static QImage wrap_in(const uint32_t *px, int w, int h, int fmt) {
    QImage img(w, h, (QImage::Format)fmt);
    for (int y = 0; y < h; y++) memcpy(img.scanLine(y), px + (size_t)y * w, (size_t)w * 4);
    return img;
}
static void copy_out(const QImage &img, uint32_t *out) {
    for (int y = 0; y < img.height(); y++)
        memcpy(out + (size_t)y * img.width(), img.constScanLine(y), (size_t)img.width() * 4);
}

extern "C" {

// kind 0: drawImage(QRectF(x, y, w, h), img [mirrored]); kind 1: fillRect(QRectF, QColor(argb));
// kind 2: translate(x + w/2, y + h/2); rotate(deg); drawImage(QRectF(-w/2, -h/2, w, h), img)
// on a cw x ch RGB32 canvas `inout`, with opacity, smooth = SmoothPixmapTransform, aa = Antialiasing.
void qtp_draw(int cw, int ch, uint32_t *inout, int kind, const uint32_t *img, int iw, int ih, int ifmt, int mirrored,
              double x, double y, double w, double h, double deg, double opacity, uint32_t argb, int smooth, int aa) {
    QImage canvas = wrap_in(inout, cw, ch, QImage::Format_RGB32);
    {
        QPainter p(&canvas);
        p.setRenderHint(QPainter::Antialiasing, aa != 0);
        p.setRenderHint(QPainter::SmoothPixmapTransform, smooth != 0);
        if (opacity != 1.0) p.setOpacity(opacity);
        if (kind == 1) {
            p.fillRect(QRectF(x, y, w, h), QColor::fromRgba(argb));
        } else {
            QImage src = wrap_in(img, iw, ih, ifmt);
            if (mirrored) src = src.mirrored(true, false);
            if (kind == 0) {
                p.drawImage(QRectF(x, y, w, h), src);
            } else {
                p.translate(x + w / 2, y + h / 2);
                p.rotate(deg);
                p.drawImage(QRectF(-w / 2, -h / 2, w, h), src);
            }
        }
    }
    copy_out(canvas, inout);
}

// jumper's compass primitives (jumper.cpp:137-177) under Antialiasing on a cw x ch RGB32 canvas:
// kind 10 drawEllipse(QRectF) with QBrush(c) + QPen(c, 1); 13 the pen only; 14 the brush only;
// 12 drawEllipse(QRect(int x, y, w, h)) with QBrush(argb, translucent) and no pen;
// 11 drawLine(QLine(int x, y, w, h)) with QPen(c, penw).
void qtp_prim(int cw, int ch, uint32_t *inout, int kind, double x, double y, double w, double h, uint32_t argb,
              int penw) {
    QImage canvas = wrap_in(inout, cw, ch, QImage::Format_RGB32);
    {
        QPainter p(&canvas);
        p.setRenderHint(QPainter::Antialiasing, true);
        p.setRenderHint(QPainter::SmoothPixmapTransform, true);
        const QColor c = QColor::fromRgba(argb);
        if (kind == 10 || kind == 13 || kind == 14) {
            if (kind == 13) p.setBrush(Qt::NoBrush);
            else p.setBrush(QBrush(c));
            if (kind == 14) p.setPen(Qt::NoPen);
            else p.setPen(QPen(c, 1));
            p.drawEllipse(QRectF(x, y, w, h));
        } else if (kind == 12) {
            p.setBrush(c);
            p.setPen(Qt::NoPen);
            p.drawEllipse(QRect((int)x, (int)y, (int)w, (int)h));
        } else if (kind == 11) {
            p.setBrush(QBrush(c));
            p.setPen(QPen(c, penw));
            p.drawLine((int)x, (int)y, (int)w, (int)h);
        }
    }
    copy_out(canvas, inout);
}

} // extern "C"
