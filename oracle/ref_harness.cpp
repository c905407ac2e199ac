// Driver for the reference-source pins (TEST INFRASTRUCTURE ONLY).
//
// Compiled together with the reference's own, unmodified sources read in place
// from /root/reference/procgen/src (randgen.cpp, entity.cpp, mazegen.cpp,
// cpp-utils.cpp) by `make -C oracle ref`; output only to oracle/_ref/ (git-ignored).
// Those translation units need neither <cheerp/client.h> nor Qt, so they build
// from their own few files.  The rest of the reference's step path does not
// (game.h includes <cheerp/client.h>, absent here) and is pinned differently
// (see oracle/procgen_oracle.h).
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>
#include "buffer.h"
#include "randgen.h"
#include "entity.h"
#include "mazegen.h"
#include "grid.h"

extern "C" {

// RandGen::serialize (randgen.cpp:100-106) through the reference's own WriteBuffer (buffer.h): in
// the fork write_int is a no-op and write_string copies the characters, so the bytes are exactly
// the std::mt19937 text after seed(seed) and `draws` randint() calls.  Returns the byte count.
int ref_randgen_text(int32_t seed, int draws, char *out, int length) {
    RandGen r;
    r.seed(seed);
    for (int i = 0; i < draws; i++) r.randint();
    WriteBuffer b(out, (size_t)length);
    r.serialize(&b);
    return (int)b.offset;
}

// successive raw 32-bit draws of the reference RandGen::randint() after seed(seed)
void ref_mt_stream(int32_t seed, uint32_t *out, int n) {
    RandGen r;
    r.seed(seed);
    for (int i = 0; i < n; i++) out[i] = (uint32_t)r.randint();
}

// same op encoding as oracle_randgen_script (procgen_oracle.c)
void ref_randgen_script(int32_t seed, const int32_t *ops, int nops, int32_t *out) {
    RandGen r;
    r.seed(seed);
    for (int i = 0; i < nops; i++) {
        int k = ops[3 * i], a = ops[3 * i + 1], b = ops[3 * i + 2];
        float f;
        switch (k) {
        case 0: out[i] = r.randint(a, b); break;
        case 1: out[i] = r.randn(a); break;
        case 2: f = r.rand01(); memcpy(&out[i], &f, 4); break;
        case 3: out[i] = r.randbool(); break;
        case 4: f = r.randrange(a / 8.0f, b / 8.0f); memcpy(&out[i], &f, 4); break;
        default: out[i] = r.randint(); break;
        }
    }
}

// Entity(x, y, vx, vy, rx, ry, type) followed by `steps` Entity::step() calls;
// fields written as 32-bit words in declaration order of the oracle's probe
// (x, y, vx, vy, rx, ry, rotation, alpha, life_time, will_erase, image_type).
void ref_entity_steps(const float *init, int type, int smart_step, float friction, float vrot, int expire_time,
                      int steps, uint32_t *out) {
    Entity e(init[0], init[1], init[2], init[3], init[4], init[5], type);
    e.smart_step = smart_step != 0;
    e.friction = friction;
    e.vrot = vrot;
    if (expire_time != 0) e.expire_time = expire_time;
    for (int s = 0; s < steps; s++) {
        e.step();
        float f[8] = {e.x, e.y, e.vx, e.vy, e.rx, e.ry, e.rotation, e.alpha};
        memcpy(out, f, 32);
        out[8] = (uint32_t)e.life_time;
        out[9] = (uint32_t)e.will_erase;
        out[10] = (uint32_t)e.image_type;
        out += 11;
    }
}

// MazeGen: seed a RandGen, build a maze of dim `maze_dim`, run `mode`
// (0 generate_maze, 1 generate_maze_no_dead_ends, 2 generate_maze_with_doors(num_doors)),
// then place_objects(start_obj, num_objs) if num_objs > 0.  Writes the grid
// (array_dim^2 ints, row-major) and returns array_dim.
int ref_mazegen(int32_t seed, int maze_dim, int mode, int num_doors, int start_obj, int num_objs, int32_t *out,
                uint32_t *next_draw) {
    RandGen r;
    r.seed(seed);
    MazeGen m(&r, maze_dim);
    if (mode == 0) m.generate_maze();
    else if (mode == 1) m.generate_maze_no_dead_ends();
    else m.generate_maze_with_doors(num_doors);
    if (num_objs > 0) m.place_objects(start_obj, num_objs);
    int n = m.grid.w;
    for (int i = 0; i < m.grid.w * m.grid.h; i++) out[i] = m.grid.data[i];
    *next_draw = (uint32_t)r.randint();
    return n;
}

// Argument evaluation order of the reference's compiler for a call with two RNG draws in its
// arguments (climber.cpp:196: add_entity(curr_x + .5, curr_y + randn(2) + 2 + .5,
// .15 * (randn(2) * 2 - 1), 0, .5, ENEMY)), compiled here with the same g++ and flags as the
// reference pins.  Writes y, vx of the entity for curr_x = 3, curr_y = 0 after seed(seed).
namespace {
struct ProbeEnt {
    float x, y, vx, vy, r;
    int type;
    ProbeEnt(float a, float b, float c, float d, float e, int t) : x(a), y(b), vx(c), vy(d), r(e), type(t) {}
};
struct ProbeGame {
    RandGen rand_gen;
    std::vector<std::shared_ptr<ProbeEnt>> entities;
    std::shared_ptr<ProbeEnt> add_entity(float x, float y, float vx, float vy, float r, int type) {
        std::shared_ptr<ProbeEnt> e(new ProbeEnt(x, y, vx, vy, r, type));
        entities.push_back(e);
        return e;
    }
};
} // namespace

void ref_climber_enemy_args(int32_t seed, float *out) {
    ProbeGame g;
    g.rand_gen.seed(seed);
    int curr_x = 3, curr_y = 0;
    auto ent = g.add_entity(curr_x + .5, curr_y + g.rand_gen.randn(2) + 2 + .5, .15 * (g.rand_gen.randn(2) * 2 - 1), 0, .5, 5);
    out[0] = ent->y;
    out[1] = ent->vx;
}

// leaper.cpp:155: road_lane_speeds.push_back(rand_sign() * rand_gen.randrange(min, max)) -- the
// operand order of a binary `*` is unspecified too; pinned here with the same compiler.
namespace {
struct ProbeLeaper {
    RandGen rand_gen;
    std::vector<float> road_lane_speeds;
    float rand_sign() {
        if (rand_gen.rand01() < 0.5) {
            return 1.0;
        } else {
            return -1.0;
        }
    }
};
} // namespace

void ref_leaper_lane_speed(int32_t seed, float lo, float hi, float *out) {
    ProbeLeaper g;
    g.rand_gen.seed(seed);
    g.road_lane_speeds.push_back(g.rand_sign() * g.rand_gen.randrange(lo, hi));
    out[0] = g.road_lane_speeds[0];
}
}

// caveflyer.cpp:235: float vel = (.1 * rand_gen.rand01() + .1) * (rand_gen.randn(2) * 2 - 1) --
// which operand of the `*` draws first, pinned with the reference's compiler and flags.
extern "C" void ref_caveflyer_enemy_vel(int32_t seed, float *out) {
    RandGen rand_gen;
    rand_gen.seed(seed);
    float vel = (.1 * rand_gen.rand01() + .1) * (rand_gen.randn(2) * 2 - 1);
    out[0] = vel;
}

// grid.h: Grid<int> resized to w x h (value-initialised: returns how many cells read 0), every cell
// set to 3 * index + 1 through set(), then per probe point: contains, get() (or -7 outside, the
// out-of-bounds object get_obj substitutes, basic-abstract-game.cpp:180-185), to_index, to_xy.
// Also pins that Grid::serialize through the fork's WriteBuffer writes no bytes.
extern "C" int ref_grid_ops(int w, int h, const int32_t *xy, int n, int32_t *out, int32_t *serialized_bytes) {
    Grid<int> g;
    g.resize(w, h);
    int zeros = 0;
    for (int i = 0; i < w * h; i++) zeros += g.get_index(i) == 0;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) g.set(x, y, 3 * g.to_index(x, y) + 1);
    for (int k = 0; k < n; k++) {
        const int x = xy[2 * k], y = xy[2 * k + 1];
        out[5 * k + 0] = g.contains(x, y);
        out[5 * k + 1] = g.contains(x, y) ? g.get(x, y) : -7;
        const int idx = g.to_index(x, y);
        out[5 * k + 2] = idx;
        int tx, ty;
        g.to_xy(idx, &tx, &ty);
        out[5 * k + 3] = tx;
        out[5 * k + 4] = ty;
    }
    std::vector<char> buf(1 << 16);
    WriteBuffer b(buf.data(), buf.size());
    g.serialize(&b);
    *serialized_bytes = (int32_t)b.offset;
    return zeros;
}
