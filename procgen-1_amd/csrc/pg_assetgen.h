// pg_assetgen.h -- AssetGen (reference assetgen.cpp:3-195) on the device: one wavefront paints one
// image, the way the reference's QPainter does: fillRect(QRectF) (opaque, alpha-200 SourceOver veil,
// transparent Source clear), drawEllipse(QRectF) with a solid brush (Qt's non-antialiased path fill:
// QBezier flattening -> QOutlineMapper 26.6 outline -> QRasterizer scan conversion) and a 1-px pen
// (QCosmeticStroker, aliased).  Used for `use_generated_assets`: the 64 x 64 sprites of every image
// type (basic-abstract-game.cpp:101-107, at make) and each env's 500 x 500 background, repainted
// with the env's rand_gen at every reset (:778-782).  Same arithmetic as the oracle's restatement
// (oracle/procgen_oracle.c ag_*, pinned against the reference's assetgen.cpp built with Qt 5.9.7).
//
// Execution model: every lane runs the painter's control flow on identical (uniform) values; the
// pixel work is lane-parallel -- spans of a fill row across lanes, the rows of an ellipse fill one
// per lane -- and the cosmetic stroker (a sequential state machine) stores from lane 0.
#pragma once
#include "pg_device.h"

#define AG_BG_DIM 500
#define AG_SPRITE_DIM 64
#define AG_FMT_RGB32 4
#define AG_FMT_ARGB32 5
#define AG_MAX_POLY 1024
#define AG_CS_MAXSUB 6

struct AgBez { double x1, y1, x2, y2, x3, y3, x4, y4; };
struct AgPtD { double x, y; };

// LDS scratch of one painting wave (uniform data: every lane writes the same value)
struct AgLds {
    int2 poly[AG_MAX_POLY];          // the flattened ellipse outline in 26.6
    AgBez bst[10];                   // QBezier::addToPolygon's subdivision stack
    int blv[10];
    AgPtD cs[3 * AG_CS_MAXSUB + 4];  // renderCubicSubdivision's point array
    int cstack[2 * AG_CS_MAXSUB + 2];
};

// Canvas + generator: Rng::next() returns the next raw mt19937 draw (uniform).
template <class Rng>
struct AgPainter {
    uint32_t *px;
    int w, h, fmt, source;
    AgLds *ls;
    Rng rng;
    int err; // bits: 1 outline overflow, 2 > 4 crossings in a row, 4 > 1 span in a row, 8 integral ellipse rect
             // (Qt's midpoint path, not restated)
};

DEV uint32_t ag_byte_mul(uint32_t x, uint32_t a) {
    uint32_t t = (x & 0xff00ffu) * a;
    t = (t + ((t >> 8) & 0xff00ffu) + 0x800080u) >> 8;
    t &= 0xff00ffu;
    x = ((x >> 8) & 0xff00ffu) * a;
    x = (x + ((x >> 8) & 0xff00ffu) + 0x800080u);
    x &= 0xff00ff00u;
    return x | t;
}
DEV uint32_t ag_div_65535(uint32_t x) { return (x + (x >> 16) + 0x8000u) >> 16; }
DEV uint32_t ag_div_257(uint32_t x) {
    x += 128u;
    return (x - (x >> 8)) >> 8;
}
// qPremultiply(QColor::rgba64()).toArgb32(): the raster engine's solid colour
DEV uint32_t ag_solid_premul(uint32_t argb) {
    const uint32_t a = (argb >> 24) * 257u;
    uint32_t out = ag_div_257(a) << 24;
    for (int s = 16; s >= 0; s -= 8) out |= ag_div_257(ag_div_65535(((argb >> s) & 255u) * 257u * a)) << s;
    return out;
}
DEV uint32_t ag_unpremultiply(uint32_t p) {
    const uint32_t a = p >> 24;
    if (a == 255) return p;
    if (a == 0) return 0;
    const uint32_t inv = (255u * 0x10000u + a / 2) / a;
    const uint32_t r = (((p >> 16) & 255u) * inv + 0x8000u) >> 16;
    const uint32_t g = (((p >> 8) & 255u) * inv + 0x8000u) >> 16;
    const uint32_t b = ((p & 255u) * inv + 0x8000u) >> 16;
    return (a << 24) | (r << 16) | (g << 8) | b;
}

// one pixel under the painter's composition mode (solid colour `pm`, premultiplied, coverage 255)
template <class P>
DEV void ag_pixel(P &p, int x, int y, uint32_t pm) {
    uint32_t *q = p.px + (size_t)y * p.w + x;
    const uint32_t a = pm >> 24;
    if (p.source || a == 255) {
        *q = p.fmt == AG_FMT_ARGB32 ? ag_unpremultiply(pm) : (pm | 0xff000000u);
    } else { // comp_func_solid_SourceOver on the premultiplied destination
        uint32_t d = *q;
        if (p.fmt == AG_FMT_ARGB32) {
            const uint32_t da = d >> 24;
            d = da == 255 ? d : (da == 0 ? 0 : (ag_byte_mul(d | 0xff000000u, da) & 0x00ffffffu) | (da << 24));
        }
        d = pm + ag_byte_mul(d, 255u - a);
        *q = p.fmt == AG_FMT_ARGB32 ? ag_unpremultiply(d) : d;
    }
}

// a coverage-255 span [x0, x1) of row y, lanes across x
template <class P>
DEV void ag_span(P &p, int y, int x0, int x1, uint32_t pm) {
    if (y < 0 || y >= p.h) return;
    if (x0 < 0) x0 = 0;
    if (x1 > p.w) x1 = p.w;
    for (int x = x0 + LANE; x < x1; x += 64) ag_pixel(p, x, y, pm);
}

// QPainter::fillRect(QRectF, QColor): toNormalizedFillRect (qRound of the edges); a transparent
// colour under SourceOver paints nothing; ARGB32 under Source / opaque: qt_rectfill_nonpremul_argb32
template <class P>
DEV void ag_fill_rectf(P &p, double x, double y, double w, double h, uint32_t argb) {
    const uint32_t pm = ag_solid_premul(argb);
    if ((pm >> 24) == 0 && !p.source) return;
    int x1 = qRound(x), y1 = qRound(y), x2 = qRound(x + w), y2 = qRound(y + h);
    if (x2 < x1) { const int t = x1; x1 = x2; x2 = t; }
    if (y2 < y1) { const int t = y1; y1 = y2; y2 = t; }
    if (y1 < 0) y1 = 0;
    if (y2 > p.h) y2 = p.h;
    if (p.fmt == AG_FMT_ARGB32 && (p.source || (pm >> 24) == 255)) {
        const uint32_t a16 = (argb >> 24) * 257u;
        uint32_t v = argb;
        if (a16 != 0 && a16 != 65535) {
            v = (argb >> 24) << 24;
            for (int sh = 16; sh >= 0; sh -= 8) {
                const uint32_t p16 = ag_div_65535(((argb >> sh) & 255u) * 257u * a16);
                v |= ag_div_257((p16 * 65535u + a16 / 2) / a16) << sh;
            }
        } else if (a16 == 0) {
            v = 0;
        }
        if (x1 < 0) x1 = 0;
        if (x2 > p.w) x2 = p.w;
        for (int yy = y1; yy < y2; yy++)
            for (int xx = x1 + LANE; xx < x2; xx += 64) p.px[(size_t)yy * p.w + xx] = v;
        return;
    }
    for (int yy = y1; yy < y2; yy++) ag_span(p, yy, x1, x2, pm);
}

// ---- drawEllipse(QRectF): QPaintEngineEx::drawEllipse -> qt_curves_for_arc(rect, 0, -360)
#define AG_KAPPA 0.5522847498
DEV void ag_ellipse_points(double x, double y, double w, double h, AgPtD pts[13]) {
    const double w2 = w / 2, w2k = w2 * AG_KAPPA, h2 = h / 2, h2k = h2 * AG_KAPPA;
    pts[0] = {x + w, y + h2};
    pts[1] = {x + w, y + h2 + h2k}; pts[2] = {x + w2 + w2k, y + h}; pts[3] = {x + w2, y + h};
    pts[4] = {x + w2 - w2k, y + h}; pts[5] = {x, y + h2 + h2k}; pts[6] = {x, y + h2};
    pts[7] = {x, y + h2 - h2k}; pts[8] = {x + w2 - w2k, y}; pts[9] = {x + w2, y};
    pts[10] = {x + w2 + w2k, y}; pts[11] = {x + w, y + h2 - h2k}; pts[12] = {x + w, y + h2};
}
// QBezier::split, in Qt's write order
DEV void ag_bez_split(const AgBez &s, AgBez &first, AgBez &second) {
    double c = (s.x2 + s.x3) * .5;
    first.x2 = (s.x1 + s.x2) * .5;
    second.x3 = (s.x3 + s.x4) * .5;
    first.x1 = s.x1;
    second.x4 = s.x4;
    first.x3 = (first.x2 + c) * .5;
    second.x2 = (second.x3 + c) * .5;
    first.x4 = second.x1 = (first.x3 + second.x2) * .5;
    c = (s.y2 + s.y3) * .5;
    first.y2 = (s.y1 + s.y2) * .5;
    second.y3 = (s.y3 + s.y4) * .5;
    first.y1 = s.y1;
    second.y4 = s.y4;
    first.y3 = (first.y2 + c) * .5;
    second.y2 = (second.y3 + c) * .5;
    first.y4 = second.y1 = (first.y3 + second.y2) * .5;
}
// QOutlineMapper's qreal_to_fixed_26_6 (qRound)
DEV int ag_fixed(double v) { return qRound(v * 64); }
// QBezier::addToPolygon(threshold 0.25), appending 26.6 end points to ls->poly from index n
template <class P>
DEV int ag_flatten(P &p, const AgBez &b0, int n) {
    AgLds *L = p.ls;
    L->bst[0] = b0;
    L->blv[0] = 9;
    int top = 0;
    while (top >= 0) {
        const AgBez b = L->bst[top];
        const double y4y1 = b.y4 - b.y1, x4x1 = b.x4 - b.x1;
        double l = fabs(x4x1) + fabs(y4y1), d;
        if (l > 1.) {
            d = fabs((x4x1) * (b.y1 - b.y2) - (y4y1) * (b.x1 - b.x2)) +
                fabs((x4x1) * (b.y1 - b.y3) - (y4y1) * (b.x1 - b.x3));
        } else {
            d = fabs(b.x1 - b.x2) + fabs(b.y1 - b.y2) + fabs(b.x1 - b.x3) + fabs(b.y1 - b.y3);
            l = 1.;
        }
        if (d < 0.25 * l || L->blv[top] == 0) {
            if (n < AG_MAX_POLY) L->poly[n] = make_int2(ag_fixed(b.x4), ag_fixed(b.y4));
            else p.err |= 1;
            n++;
            top--;
        } else {
            AgBez first, second;
            ag_bez_split(b, first, second);
            const int lv = L->blv[top] - 1;
            L->bst[top] = second;
            L->blv[top] = lv;
            L->bst[top + 1] = first;
            L->blv[top + 1] = lv;
            top++;
        }
    }
    return n;
}

// QScanConverter (QRasterizer, no legacy rounding): the crossing of one outline edge with scan row y,
// clipped to [leftFP, rightFP] as QScanConverter::clip replaces the out-of-range parts with
// vertical lines at the edge.  Returns false when the edge does not cover row y.
DEV bool ag_edge_x(int ax, int ay, int bx, int by, int y, int top, int bottom, int leftFP, int rightFP, int &x,
                   int &wind) {
    int winding = 1;
    if (ay > by) {
        int t = ax; ax = bx; bx = t;
        t = ay; ay = by; by = t;
        winding = -1;
    }
    int iTop = (ay + 32) >> 6, iBottom = (by - 32) >> 6;
    if (iTop < top) iTop = top;
    if (iBottom > bottom) iBottom = bottom;
    if (y < iTop || y > iBottom) return false;
    wind = winding;
    const int aFP = 65536 / 2 + ax * 1024;
    if (bx == ax) {
        x = (aFP < leftFP ? leftFP : (aFP > rightFP ? rightFP : aFP)) >> 16;
        return true;
    }
    const double slope = (double)(bx - ax) / (double)(by - ay);
    const int slopeFP = (int)(slope * 65536.);
    int xFP = aFP + (int)(((int64_t)slopeFP * ((int64_t)iTop * 65536 + 65536 / 2 - (int64_t)ay * 1024)) >> 16);
    // the two clips in order (left, then right), each possibly splitting the line
    for (int e = 0; e < 2; e++) {
        const int edgeFP = e == 0 ? leftFP : rightFP;
        const bool right = e == 1;
        if (xFP == edgeFP) {
            if ((slopeFP > 0) ^ right) continue;
            x = edgeFP >> 16; // the whole remaining line is the edge
            return true;
        }
        const int lastFP = xFP + slopeFP * (iBottom - iTop);
        if (lastFP == edgeFP) {
            if ((slopeFP < 0) ^ right) continue;
            x = edgeFP >> 16;
            return true;
        }
        if ((lastFP < edgeFP) ^ (xFP < edgeFP)) {
            const int deltaY = (int)((edgeFP - xFP) / (slopeFP / 65536.));
            if ((xFP < edgeFP) ^ right) { // the top part is clipped
                const int iHeight = (deltaY + 1) >> 16;
                const int iMiddle = iTop + iHeight;
                if (y <= iMiddle) {
                    x = edgeFP >> 16;
                    return true;
                }
                if (iMiddle == iBottom) return false; // (unreachable: y <= iBottom)
                xFP += slopeFP * (iHeight + 1);
                iTop = iMiddle + 1;
            } else { // the bottom part is clipped
                const int iHeight = deltaY >> 16;
                const int iMiddle = iTop + iHeight;
                if (iMiddle != iBottom) {
                    if (y > iMiddle) {
                        x = edgeFP >> 16;
                        return true;
                    }
                    iBottom = iMiddle;
                }
            }
        } else if ((xFP < edgeFP) ^ right) {
            x = edgeFP >> 16;
            return true;
        }
    }
    x = (int)(((int64_t)xFP + (int64_t)slopeFP * (y - iTop)) >> 16);
    return true;
}

// the brush: rows one per lane; each lane collects its row's crossings (winding fill), the wave then
// paints the 64 rows' spans across lanes
template <class P>
DEV void ag_fill_ellipse(P &p, const AgPtD pts[13], uint32_t pm) {
    int n = 0;
    p.ls->poly[0] = make_int2(ag_fixed(pts[0].x), ag_fixed(pts[0].y));
    n = 1;
    AgPtD last = pts[0];
    for (int k = 0; k < 4; k++) {
        AgBez b = {last.x, last.y, pts[3 * k + 1].x, pts[3 * k + 1].y, pts[3 * k + 2].x, pts[3 * k + 2].y,
                   pts[3 * k + 3].x, pts[3 * k + 3].y};
        // the last appended point of the previous curve is its end point pts[3k] (bit-identical)
        n = ag_flatten(p, b, n);
        last = pts[3 * k + 3];
    }
    if (n > AG_MAX_POLY) return;
    int miny = 0x7fffffff, maxy = -0x7fffffff;
    for (int i = LANE; i < n; i += 64) {
        miny = min(miny, p.ls->poly[i].y);
        maxy = max(maxy, p.ls->poly[i].y);
    }
    for (int o = 32; o > 0; o >>= 1) {
        miny = min(miny, __shfl_xor(miny, o));
        maxy = max(maxy, __shfl_xor(maxy, o));
    }
    int top = (miny + 32) >> 6, bottom = (maxy - 32) >> 6;
    if (top < 0) top = 0;
    if (bottom > p.h - 1) bottom = p.h - 1;
    const int leftFP = 0, rightFP = p.w * 65536;
    for (int y0 = top; y0 <= bottom; y0 += 64) {
        const int y = y0 + LANE;
        int sx0 = 0, sx1 = 0; // this lane's row span (the convex outline crosses a row twice)
        if (y <= bottom) {
            int xs[4], ws[4], k = 0;
            for (int i = 0; i + 1 < n; i++) {
                int x, wd;
                const int2 a = p.ls->poly[i], b = p.ls->poly[i + 1];
                if (!ag_edge_x(a.x, a.y, b.x, b.y, y, top, bottom, leftFP, rightFP, x, wd)) continue;
                if (k < 4) {
                    int j = k++;
                    while (j > 0 && xs[j - 1] > x) { xs[j] = xs[j - 1]; ws[j] = ws[j - 1]; j--; }
                    xs[j] = x;
                    ws[j] = wd;
                } else {
                    p.err |= 2;
                }
            }
            int x = 0, wind = 0, spans = 0;
            for (int i = 0; i < k; i++) {
                if (wind != 0 && xs[i] > x) {
                    if (spans++ == 0) { sx0 = x; sx1 = xs[i]; }
                    else p.err |= 4;
                }
                x = xs[i];
                wind += ws[i];
            }
        }
        for (int o = 32; o > 0; o >>= 1) p.err |= __shfl_xor(p.err, o);
        const int rows = min(64, bottom - y0 + 1);
        for (int r = 0; r < rows; r++) {
            const int a = __builtin_amdgcn_readlane(sx0, r), b = __builtin_amdgcn_readlane(sx1, r);
            if (b > a) ag_span(p, y0 + r, a, b, pm);
        }
    }
}

// ---- QCosmeticStroker (aliased, solid, no dash) for a 1-px pen
enum { AG_T2B = 1, AG_B2T = 2, AG_L2R = 4, AG_R2L = 8, AG_VMASK = 3, AG_HMASK = 12 };
enum { AG_CAPBEGIN = 1, AG_CAPEND = 2 };
struct AgStroker {
    uint32_t pm;
    double xmin, xmax, ymin, ymax;
    int lastx, lasty, lastDir;
    bool lastAxisAligned;
};
#define AG_INT_MIN (-2147483647 - 1)
DEV int ag_f26(double v) { return (int)(v * 64.); }
DEV int ag_fdiv(int x, int y) {
    if (abs(x) > 0x7fff) return (int)(((int64_t)x * 65536) / y);
    return x * 65536 / y;
}
DEV int ag_swap_caps(int caps) { return ((caps & 1) << 1) | ((caps & 2) >> 1); }
DEV void ag_cap_adjust(int caps, int &x1, int &x2, int &y, int yinc) {
    if (caps & AG_CAPBEGIN) {
        x1 -= 32;
        y -= yinc >> 1;
    }
    if (caps & AG_CAPEND) x2 += 32;
}
template <class P>
DEV void ag_cs_pixel(P &p, const AgStroker &s, int x, int y) {
    if (x < 0 || x >= p.w || y < 0 || y >= p.h) return;
    if (LANE == 0) ag_pixel(p, x, y, s.pm);
}
// QCosmeticStroker::clipLine: true = completely outside
DEV bool ag_cs_clip(AgStroker &s, double &x1, double &y1, double &x2, double &y2) {
    if (x1 < s.xmin) {
        if (x2 <= s.xmin) goto clipped;
        y1 += (y2 - y1) / (x2 - x1) * (s.xmin - x1);
        x1 = s.xmin;
    } else if (x1 > s.xmax) {
        if (x2 >= s.xmax) goto clipped;
        y1 += (y2 - y1) / (x2 - x1) * (s.xmax - x1);
        x1 = s.xmax;
    }
    if (x2 < s.xmin) {
        s.lastx = AG_INT_MIN;
        y2 += (y2 - y1) / (x2 - x1) * (s.xmin - x2);
        x2 = s.xmin;
    } else if (x2 > s.xmax) {
        s.lastx = AG_INT_MIN;
        y2 += (y2 - y1) / (x2 - x1) * (s.xmax - x2);
        x2 = s.xmax;
    }
    if (y1 < s.ymin) {
        if (y2 <= s.ymin) goto clipped;
        x1 += (x2 - x1) / (y2 - y1) * (s.ymin - y1);
        y1 = s.ymin;
    } else if (y1 > s.ymax) {
        if (y2 >= s.ymax) goto clipped;
        x1 += (x2 - x1) / (y2 - y1) * (s.ymax - y1);
        y1 = s.ymax;
    }
    if (y2 < s.ymin) {
        s.lastx = AG_INT_MIN;
        x2 += (x2 - x1) / (y2 - y1) * (s.ymin - y2);
        y2 = s.ymin;
    } else if (y2 > s.ymax) {
        s.lastx = AG_INT_MIN;
        x2 += (x2 - x1) / (y2 - y1) * (s.ymax - y2);
        y2 = s.ymax;
    }
    return false;
clipped:
    s.lastx = AG_INT_MIN;
    return true;
}
// drawLine<drawPixel, NoDasher>, both branches (vert: major axis y): a reversal caps the new
// segment's path-start end (CapEnd swapped, CapBegin otherwise, a CapBegin that rounds one pixel
// before lastPixel rounded back); the same-direction dropout test reads |dx| <= 1 && |dy| > 1 in
// both branches (oracle cs_run)
template <class P>
DEV void ag_cs_run(P &p, AgStroker &s, bool vert, int a1, int b1, int a2, int b2, int caps) {
    int dir = vert ? AG_T2B : AG_L2R;
    bool swapped = false;
    if (a1 > a2) {
        swapped = true;
        int t = a1; a1 = a2; a2 = t;
        t = b1; b1 = b2; b2 = t;
        caps = ag_swap_caps(caps);
        dir = vert ? AG_B2T : AG_R2L;
    }
    const int binc = ag_fdiv(b2 - b1, a2 - a1);
    int b = b1 * 1024;
    if ((s.lastDir ^ (vert ? AG_VMASK : AG_HMASK)) == dir) caps |= swapped ? AG_CAPEND : AG_CAPBEGIN;
    ag_cap_adjust(caps, a1, a2, b, binc);
    const int round = (binc > 0) ? 32 : 0;
    int a = (a1 + 32) >> 6;
    int as = (a2 + 32) >> 6;
    if ((caps & AG_CAPBEGIN) && (vert ? s.lasty : s.lastx) == a + 1) a++; // CapBegin rounded back
    int lx = s.lastx, ly = s.lasty;
    if (a != as) {
        b += ((a * 64) + round - a1) * binc >> 6;
        int fa = a, fb = b >> 16;
        int la = as - 1, lb = (b + (as - a - 1) * binc) >> 16;
        if (swapped) {
            int t = fa; fa = la; la = t;
            t = fb; fb = lb; lb = t;
        }
        const int fx = vert ? fb : fa, fy = vert ? fa : fb;
        lx = vert ? lb : la;
        ly = vert ? la : lb;
        const bool axisAligned = abs(binc) < (1 << 14);
        if (s.lastx > -1) {
            if (fx == s.lastx && fy == s.lasty) {
                if (swapped) --as;
                else { ++a; b += binc; }
            } else if (s.lastDir != dir && (((axisAligned && s.lastAxisAligned) && s.lastx != fx && s.lasty != fy) ||
                                            (abs(s.lastx - fx) > 1 || abs(s.lasty - fy) > 1))) {
                if (swapped) ++as;
                else { --a; b -= binc; }
            } else if (s.lastDir == dir && abs(s.lastx - fx) <= 1 && abs(s.lasty - fy) > 1) {
                b += binc >> 1;
                const int nl = swapped ? (b >> 16) : ((b + (as - a - 1) * binc) >> 16);
                if (vert) lx = nl;
                else ly = nl;
            }
        }
        s.lastDir = dir;
        s.lastAxisAligned = axisAligned;
        do {
            if (vert) ag_cs_pixel(p, s, b >> 16, a);
            else ag_cs_pixel(p, s, a, b >> 16);
            b += binc;
        } while (++a < as);
    }
    s.lastx = lx;
    s.lasty = ly;
}
template <class P>
DEV void ag_cs_line(P &p, AgStroker &s, double rx1, double ry1, double rx2, double ry2, int caps) {
    if (ag_cs_clip(s, rx1, ry1, rx2, ry2)) return;
    const int x1 = ag_f26(rx1), y1 = ag_f26(ry1), x2 = ag_f26(rx2), y2 = ag_f26(ry2);
    const int dx = abs(x2 - x1), dy = abs(y2 - y1);
    if (dx < dy) ag_cs_run(p, s, true, y1, x1, y2, x2, caps);
    else if (dx) ag_cs_run(p, s, false, x1, y1, x2, y2, caps);
}
// QCosmeticStroker::calculateLastPoint (Qt 5.9 keeps lastDir when the closing segment has no pixel)
DEV void ag_cs_last_point(AgStroker &s, double rx1, double ry1, double rx2, double ry2) {
    s.lastx = AG_INT_MIN;
    s.lasty = AG_INT_MIN;
    if (ag_cs_clip(s, rx1, ry1, rx2, ry2)) return;
    int x1 = ag_f26(rx1), y1 = ag_f26(ry1), x2 = ag_f26(rx2), y2 = ag_f26(ry2);
    const int dx = abs(x2 - x1), dy = abs(y2 - y1);
    const bool vert = dx < dy;
    if (!vert && !dx) return;
    int a1 = vert ? y1 : x1, b1 = vert ? x1 : y1, a2 = vert ? y2 : x2, b2 = vert ? x2 : y2;
    bool swapped = false;
    if (a1 > a2) {
        swapped = true;
        int t = a1; a1 = a2; a2 = t;
        t = b1; b1 = b2; b2 = t;
    }
    const int binc = ag_fdiv(b2 - b1, a2 - a1);
    int b = b1 * 1024;
    const int a = (a1 + 32) >> 6, as = (a2 + 32) >> 6;
    const int round = (binc > 0) ? 32 : 0;
    if (a != as) {
        b += ((a * 64) + round - a1) * binc >> 6;
        int pa, pb;
        if (swapped) {
            pa = a;
            pb = b >> 16;
            s.lastDir = vert ? AG_B2T : AG_R2L;
        } else {
            pa = as - 1;
            pb = (b + (as - a - 1) * binc) >> 16;
            s.lastDir = vert ? AG_T2B : AG_L2R;
        }
        s.lastx = vert ? pb : pa;
        s.lasty = vert ? pa : pb;
        s.lastAxisAligned = abs(binc) < (1 << 14);
    }
}
// splitCubic (points[3] = start, points[0] = end; the first half goes to points[3..6])
DEV void ag_cs_split(AgPtD *q) {
    const double half = .5;
    double a, b, c, d;
    q[6].x = q[3].x;
    c = q[1].x;
    d = q[2].x;
    q[1].x = a = (q[0].x + c) * half;
    q[5].x = b = (q[3].x + d) * half;
    c = (c + d) * half;
    q[2].x = a = (a + c) * half;
    q[4].x = b = (b + c) * half;
    q[3].x = (a + b) * half;
    q[6].y = q[3].y;
    c = q[1].y;
    d = q[2].y;
    q[1].y = a = (q[0].y + c) * half;
    q[5].y = b = (q[3].y + d) * half;
    c = (c + d) * half;
    q[2].y = a = (a + c) * half;
    q[4].y = b = (b + c) * half;
    q[3].y = (a + b) * half;
}
// renderCubic -> renderCubicSubdivision, the recursion unrolled onto an (offset, level) stack
template <class P>
DEV void ag_cs_cubic(P &p, AgStroker &s, AgPtD p1, AgPtD p2, AgPtD p3, AgPtD p4) {
    AgPtD *q = p.ls->cs;
    int *st = p.ls->cstack;
    q[3] = p1;
    q[2] = p2;
    q[1] = p3;
    q[0] = p4;
    int sp = 0;
    st[0] = 0 | (AG_CS_MAXSUB << 8); // offset | level << 8
    while (sp >= 0) {
        const int off = st[sp] & 0xff, level = st[sp] >> 8;
        sp--;
        AgPtD *pts = q + off;
        if (level) {
            const double dx = pts[3].x - pts[0].x, dy = pts[3].y - pts[0].y;
            const double len = ((double).25) * (fabs(dx) + fabs(dy));
            if (fabs(dx * (pts[0].y - pts[2].y) - dy * (pts[0].x - pts[2].x)) >= len ||
                fabs(dx * (pts[0].y - pts[1].y) - dy * (pts[0].x - pts[1].x)) >= len) {
                ag_cs_split(pts);
                // renderCubicSubdivision(points + 3, level - 1); then (points, level - 1)
                st[++sp] = off | ((level - 1) << 8);
                st[++sp] = (off + 3) | ((level - 1) << 8);
                continue;
            }
        }
        ag_cs_line(p, s, pts[3].x, pts[3].y, pts[0].x, pts[0].y, 0);
    }
}
// QCosmeticStroker::drawPath of the ellipse's closed subpath (no caps; the closing segment, cp2 ->
// end of the last curve, primes lastPixel / lastDir; the stroker starts with lastDir LeftToRight)
template <class P>
DEV void ag_stroke_ellipse(P &p, const AgPtD pts[13], uint32_t pm) {
    AgStroker s;
    s.pm = pm;
    s.xmin = -1;
    s.xmax = p.w + 1;
    s.ymin = -1;
    s.ymax = p.h + 1;
    s.lastAxisAligned = false;
    s.lastDir = AG_L2R;
    s.lastx = AG_INT_MIN;
    s.lasty = AG_INT_MIN;
    ag_cs_last_point(s, pts[11].x, pts[11].y, pts[12].x, pts[12].y);
    for (int k = 0; k < 4; k++) ag_cs_cubic(p, s, pts[3 * k], pts[3 * k + 1], pts[3 * k + 2], pts[3 * k + 3]);
    wave_sync(); // lane 0's stores before the next primitive's lane-parallel ones
}

// setBrush(QBrush(c1)); setPen(QPen(c2)); drawEllipse(QRectF) (assetgen.cpp:95-99)
template <class P>
DEV void ag_draw_ellipse(P &p, double x, double y, double w, double h, uint32_t brush, uint32_t pen) {
    if (w <= 0 || h <= 0) return;
    if (x == (double)(int)x && y == (double)(int)y && w == (double)(int)w && h == (double)(int)h) {
        p.err |= 8; // QRasterPaintEngine::drawEllipse's midpoint path (not restated)
        return;
    }
    AgPtD pts[13];
    ag_ellipse_points(x, y, w, h, pts);
    ag_fill_ellipse(p, pts, ag_solid_premul(brush));
    wave_sync();
    ag_stroke_ellipse(p, pts, ag_solid_premul(pen));
}

// ---- AssetGen (assetgen.cpp:3-195); float / double promotion as the C++ source has it
template <class P>
DEV float ag_rand01(P &p) { return rg_rand01_of(p.rng.next()); }
template <class P>
DEV bool ag_randbool(P &p) { return (double)ag_rand01(p) > .5; }

struct AgColorGen {
    float rgb_start[3], rgb_len[3];
};
template <class P>
DEV void ag_roll(P &p, AgColorGen &g) { // :10-20
    for (int i = 0; i < 3; i++) g.rgb_len[i] = ag_rand01(p);
    for (int i = 0; i < 3; i++) g.rgb_start[i] = ag_rand01(p) * (1 - g.rgb_len[i]);
    (void)ag_rand01(p); // p_rect
}
template <class P>
DEV uint32_t ag_rand_color(P &p, const AgColorGen &g) { // :22-28
    uint32_t c = 0xff000000u;
    for (int i = 0; i < 3; i++) c |= (uint32_t)(int)(255 * (ag_rand01(p) * g.rgb_len[i] + g.rgb_start[i])) << (16 - 8 * i);
    return c;
}
struct AgRect { double x, y, w, h; };
template <class P>
DEV AgRect ag_choose_sub_rect(P &p, AgRect rect, float min_dim, float max_dim) { // :35-51
    const int w = (int)rect.w, h = (int)rect.h;
    const int smaller = (w > h) ? h : w;
    const float del_dim = max_dim - min_dim;
    const float rdx = (ag_rand01(p) * del_dim + min_dim) * smaller;
    const float rdy = (ag_rand01(p) * del_dim + min_dim) * smaller;
    const float rx_off = ag_rand01(p) * (w - rdx);
    const float ry_off = ag_rand01(p) * (h - rdy);
    return {rx_off + rect.x, ry_off + rect.y, (double)rdx, (double)rdy};
}
template <class P>
DEV void ag_paint_shape(P &p, AgRect main_rect, const AgColorGen &cg) { // :75-102 (split_rect :53-73)
    const int k = rg_randn_of(p.rng.next(), 10);
    const int num_splits = (k * k) / 50 + 1;
    const bool is_horizontal = ag_randbool(p);
    const float x = (float)main_rect.x, y = (float)main_rect.y, w = (float)main_rect.w, h = (float)main_rect.h;
    const float dw = w / num_splits, dh = h / num_splits;
    const bool use_rect = ag_randbool(p);
    const bool regen_colors = ag_randbool(p);
    uint32_t c1 = ag_rand_color(p, cg);
    uint32_t c2 = ag_rand_color(p, cg);
    for (int i = 0; i < num_splits; i++) {
        AgRect r;
        if (is_horizontal) r = {(double)(x + i * dw), (double)y, (double)dw, (double)h};
        else r = {(double)x, (double)(y + i * dh), (double)w, (double)dh};
        if (regen_colors) {
            c1 = ag_rand_color(p, cg);
            c2 = ag_rand_color(p, cg);
        }
        if (use_rect) ag_fill_rectf(p, r.x, r.y, r.w, r.h, c1);
        else ag_draw_ellipse(p, r.x, r.y, r.w, r.h, c1, c2);
        wave_sync();
    }
}
// paint_rect_resource (:104-132); the recursion is at most one level deep (num_recurse <= 1)
template <int DEPTH, class P>
DEV void ag_paint_rect_resource(P &p, AgRect rect, int num_recurse, int blotch_scale) {
    AgColorGen cg;
    ag_roll(p, cg);
    const uint32_t bgcolor = ag_rand_color(p, cg);
    ag_fill_rectf(p, rect.x, rect.y, rect.w, rect.h, bgcolor);
    wave_sync();
    const float scale = (float)(.3 + .7 * (double)ag_rand01(p));
    const float max_rand_dim = (float)(.5 * (double)scale);
    const float min_rand_dim = (float)(.05 * (double)scale);
    const int num_blotches = rg_randint_of(p.rng.next(), blotch_scale, 2 * blotch_scale);
    const float p_recurse = (float)((double)ag_rand01(p) * .75);
    for (int j = 0; j < num_blotches; j++) {
        const AgRect dst3 = ag_choose_sub_rect(p, rect, min_rand_dim, max_rand_dim);
        bool rec = false;
        if constexpr (DEPTH > 0) rec = (num_recurse > 0) && (ag_rand01(p) < p_recurse);
        if (rec) {
            if constexpr (DEPTH > 0) ag_paint_rect_resource<DEPTH - 1>(p, dst3, num_recurse - 1, 10);
        } else {
            ag_paint_shape(p, dst3, cg);
        }
    }
    ag_fill_rectf(p, rect.x, rect.y, rect.w, rect.h, (bgcolor & 0x00ffffffu) | (200u << 24)); // setAlpha(200)
    wave_sync();
}
template <class P>
DEV AgRect ag_create_bar(P &p, AgRect rect, bool is_horizontal) { // :134-149
    const float k1 = (float)(.45 + (double)ag_rand01(p) * .4);
    const float k2 = (float)(.45 + (double)ag_rand01(p) * .4);
    const float w = (float)(rect.w * k1 * k1);
    const float h = (float)(rect.h * k2 * k2);
    const float pct = ag_rand01(p);
    if (is_horizontal == 0) return {0, (rect.h - h) * pct, rect.w, (double)h};
    return {(rect.h - w) * pct, 0, (double)w, rect.h}; // the reference uses height() for x
}
template <class P>
DEV void ag_paint_shape_resource(P &p, AgRect rect) { // :151-184
    AgColorGen cg;
    ag_roll(p, cg);
    const bool horizontal_first = ag_randbool(p);
    const int nbar1 = rg_randn_of(p.rng.next(), 3) / 2 + 1;
    const int nbar2 = rg_randn_of(p.rng.next(), 3) / 2 + 1;
    const int saved = p.source;
    p.source = 1; // save(); setCompositionMode(CompositionMode_Source)
    ag_fill_rectf(p, rect.x, rect.y, rect.w, rect.h, 0x00000000u);
    wave_sync();
    for (int i = 0; i < nbar1; i++) ag_paint_shape(p, ag_create_bar(p, rect, horizontal_first), cg);
    for (int i = 0; i < nbar2; i++) ag_paint_shape(p, ag_create_bar(p, rect, !horizontal_first), cg);
    const int num_blotches = rg_randint_of(p.rng.next(), 1, 5);
    for (int j = 0; j < num_blotches; j++) ag_paint_shape(p, ag_choose_sub_rect(p, rect, 0.1f, 0.6f), cg);
    p.source = saved; // restore()
}
// AssetGen::generate_resource (:186-195)
template <class P>
DEV void ag_generate_resource(P &p, int num_recurse, int blotch_scale, bool is_rect) {
    const AgRect rect = {0, 0, (double)p.w, (double)p.h};
    if (is_rect) ag_paint_rect_resource<1>(p, rect, num_recurse, blotch_scale);
    else ag_paint_shape_resource(p, rect);
}

// use_block_asset(type) of each game (basic-abstract-game.cpp:412-414 and the games' overrides:
// caveflyer.cpp:81, chaser.cpp:74, climber.cpp:128, coinrun.cpp:183, dodgeball.cpp:153,
// fruitbot.cpp:137, heist.cpp:62, jumper.cpp:107, leaper.cpp:87, ninja.cpp:135)
static inline __host__ __device__ bool ag_use_block_asset(int game, int t) {
    switch (game) {
    case PG_GAME_CAVEFLYER: return t == 8;                       // CAVEWALL
    case PG_GAME_CHASER: return t == 5;                          // MAZE_WALL
    case PG_GAME_CLIMBER: case PG_GAME_COINRUN: return t == 15 || t == 16; // WALL_MID, WALL_TOP
    case PG_GAME_DODGEBALL: return t == 1 || t == 5 || t == 7;   // LAVA_WALL, DOOR, DOOR_OPEN
    case PG_GAME_FRUITBOT: return t == 1 || t == 10 || t == 12;  // BARRIER, LOCKED_DOOR, PRESENT
    case PG_GAME_HEIST: return t == 51 || t == 1;                // WALL_OBJ, LOCKED_DOOR
    case PG_GAME_JUMPER: return t == 6 || t == 7;                // CAVEWALL, CAVEWALL_TOP
    case PG_GAME_LEAPER: return t == 3 || t == 2;                // WATER, ROAD
    case PG_GAME_NINJA: return t == 20;                          // WALL_MID
    default: return false;
    }
}
