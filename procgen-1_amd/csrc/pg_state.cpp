// pg_state.cpp -- the upstream get_state / set_state byte format (host side).
//
// The fork stubs its WriteBuffer / ReadBuffer (buffer.h:28-34, 95-115: write_int and write_float
// are no-ops, read_int returns 0), so its get_state emits only the strings and its set_state dies
// on fassert(game_name == read_string()) (game.cpp:259).  This file writes and reads the format
// the same serialize / deserialize functions define with the buffer's commented-out 4-byte
// little-endian writes in place -- upstream procgen's format: int / float = 4 bytes, bool = int,
// string = int length + bytes, vector = int count + elements, END_OF_BUFFER = 0xCAFECAFE.
//
// Members that live only in the reference's objects are produced the way the reference produces
// them: the render members (center_x / y, unit, view_dim, x_off, y_off, the drawn visibility)
// restate prepare_for_drawing(64) of the last observe (basic-abstract-game.cpp:828-847 with
// choose_center, climber.cpp:261-265, fruitbot.cpp:141-145); constants are the values the game's
// reset assigns (bossfight.cpp:218-248, fruitbot.cpp:36-37); chaser's free_cells / is_space_vec
// are the non-MAZE_WALL cells (chaser.cpp:246-257; walls never change after the reset);
// fixed_asset_seed is hash_str_uint32(name) (vecgame.cpp:156-167, 370-375); asset_rand_gen is
// never seeded without generated assets (a default std::mt19937).
#include "pg_state.h"

#include <string.h>

#include <random>
#include <sstream>

namespace {

const int32_t END_OF_BUFFER = (int32_t)0xCAFECAFE;
const int SERIALIZE_VERSION = 0; // game.cpp:6

const char *NAMES[PG_NUM_GAMES] = {"bigfish", "bossfight", "caveflyer", "chaser", "climber", "coinrun",
                                   "dodgeball", "fruitbot", "heist", "jumper", "leaper", "maze",
                                   "miner", "ninja", "plunder", "starpilot"};

// entity flags (pg_engine.h)
bool flag(int32_t f, int bit) { return (f & bit) != 0; }

struct StateWriter {
    std::vector<char> &o;
    void raw(const void *p, size_t n) { o.insert(o.end(), (const char *)p, (const char *)p + n); }
    void i(int32_t v) { raw(&v, 4); }
    void f(float v) { raw(&v, 4); }
    void b(bool v) { i(v ? 1 : 0); }
    void s(const std::string &v) {
        i((int32_t)v.size());
        raw(v.data(), v.size());
    }
};

struct StateReader {
    const char *p;
    size_t n, off;
    bool ok;
    bool need(size_t k) {
        if (!ok || off + k > n) ok = false;
        return ok;
    }
    int32_t i() {
        int32_t v = 0;
        if (need(4)) memcpy(&v, p + off, 4), off += 4;
        return v;
    }
    float f() {
        float v = 0;
        if (need(4)) memcpy(&v, p + off, 4), off += 4;
        return v;
    }
    bool b() { return i() != 0; }
    std::string s() {
        int32_t k = i();
        if (k < 0 || !need((size_t)k)) {
            ok = false;
            return std::string();
        }
        std::string v(p + off, (size_t)k);
        off += (size_t)k;
        return v;
    }
    // vector count, bounded so a corrupt count cannot run away
    int32_t count(int32_t maxn) {
        int32_t k = i();
        if (k < 0 || k > maxn) ok = false;
        return ok ? k : 0;
    }
};

float fbits(int32_t b) {
    float x;
    memcpy(&x, &b, 4);
    return x;
}
int32_t bitsf(float x) {
    int32_t b;
    memcpy(&b, &x, 4);
    return b;
}

uint32_t hash_str_uint32(const std::string &str) { // FNV-1a, vecgame.cpp:156-167
    uint32_t hash = 0x811c9dc5u;
    for (size_t i = 0; i < str.size(); i++) {
        hash = hash ^ (uint8_t)str[i];
        hash *= 0x1000193u;
    }
    return hash;
}

// prepare_for_drawing(64) of the last observe: center_x, center_y, visibility, unit, view_dim, x_off, y_off
struct ViewM { float cx, cy, vis, unit, view_dim, x_off, y_off; };
ViewM view_members(const HostEnv &h) {
    const PGEnv &s = h.s;
    float ax, ay, ary;
    if (s.agent_erased || s.num_ents <= 0) {
        ax = s.ghost_x; ay = s.ghost_y; ary = s.ghost_ry;
    } else {
        ax = fbits(h.ent[F_X][0]); ay = fbits(h.ent[F_Y][0]); ary = fbits(h.ent[F_RY][0]);
    }
    ViewM m;
    m.cx = (float)(s.main_width * .5);
    m.cy = (float)(s.main_height * .5);
    m.vis = s.visibility;
    if (s.opt_center_agent) {
        if (s.game_id == PG_GAME_CLIMBER || s.game_id == PG_GAME_FRUITBOT) {
            const float k = s.game_id == PG_GAME_CLIMBER ? 5 * ary : 2 * ary;
            m.cx = (float)(s.main_width / 2.0);
            m.cy = (float)((double)ay + s.main_width / 2.0 - (double)k);
            m.vis = (float)s.main_width;
        } else {
            m.cx = ax;
            m.cy = ay;
        }
    } else {
        m.vis = (float)(s.main_width > s.main_height ? s.main_width : s.main_height);
        if (m.vis < s.min_visibility) m.vis = s.min_visibility;
    }
    const float raw_unit = 64 / m.vis;
    m.unit = (float)((double)raw_unit * (64 / 64.0));
    m.view_dim = (float)(64.0 / (double)raw_unit);
    m.x_off = m.unit * (m.cx - m.view_dim / 2);
    m.y_off = m.unit * (m.cy - m.view_dim / 2);
    return m;
}

void write_entity(StateWriter &w, const std::vector<int32_t> *pl, size_t k) { // Entity::serialize (entity.cpp:90-134)
    auto F = [&](int f) { return fbits(pl[f][k]); };
    auto I = [&](int f) { return pl[f][k]; };
    const int32_t fl = I(F_FLAGS);
    w.f(F(F_X)); w.f(F(F_Y)); w.f(F(F_VX)); w.f(F(F_VY)); w.f(F(F_RX)); w.f(F(F_RY));
    w.i(I(F_TYPE)); w.i(I(F_IMAGE_TYPE)); w.i(I(F_IMAGE_THEME)); w.i(I(F_RENDER_Z));
    w.i(flag(fl, EF_WILL_ERASE)); w.i(flag(fl, EF_COLLIDES));
    w.f(F(F_COLLISION_MARGIN)); w.f(F(F_ROTATION)); w.f(F(F_VROT));
    w.i(flag(fl, EF_REFLECTED)); w.i(I(F_FIRE_TIME)); w.i(I(F_SPAWN_TIME)); w.i(I(F_LIFE_TIME));
    w.i(I(F_EXPIRE_TIME)); w.i(flag(fl, EF_ABS_COORDS));
    w.f(F(F_FRICTION)); w.i(flag(fl, EF_SMART_STEP)); w.i(flag(fl, EF_AVOIDS)); w.i(flag(fl, EF_AUTO_ERASE));
    w.f(F(F_ALPHA)); w.f(F(F_HEALTH)); w.f(F(F_THETA)); w.f(F(F_GROW_RATE)); w.f(F(F_ALPHA_DECAY));
    w.f(F(F_CLIMBER_SPAWN_X));
}

void read_entity(StateReader &r, std::vector<int32_t> *pl, size_t k) { // Entity::deserialize (entity.cpp:136-179)
    auto F = [&](int f) { pl[f][k] = bitsf(r.f()); };
    auto I = [&](int f) { pl[f][k] = r.i(); };
    int32_t fl = 0;
    auto B = [&](int bit) { if (r.i()) fl |= bit; };
    F(F_X); F(F_Y); F(F_VX); F(F_VY); F(F_RX); F(F_RY);
    I(F_TYPE); I(F_IMAGE_TYPE); I(F_IMAGE_THEME); I(F_RENDER_Z);
    B(EF_WILL_ERASE); B(EF_COLLIDES);
    F(F_COLLISION_MARGIN); F(F_ROTATION); F(F_VROT);
    B(EF_REFLECTED); I(F_FIRE_TIME); I(F_SPAWN_TIME); I(F_LIFE_TIME); I(F_EXPIRE_TIME); B(EF_ABS_COORDS);
    F(F_FRICTION); B(EF_SMART_STEP); B(EF_AVOIDS); B(EF_AUTO_ERASE);
    F(F_ALPHA); F(F_HEALTH); F(F_THETA); F(F_GROW_RATE); F(F_ALPHA_DECAY); F(F_CLIMBER_SPAWN_X);
    pl[F_FLAGS][k] = fl;
}

void write_randgen(StateWriter &w, const uint32_t *words, int pos) { // RandGen::serialize (randgen.cpp:100-106)
    w.i(1); // is_seeded: both generators are seeded before any state exists
    w.s(pg_mt_text(words, pos));
}

bool read_randgen(StateReader &r, uint32_t *words, int32_t &pos) {
    r.i(); // is_seeded
    int p = 0;
    const std::string t = r.s();
    if (!r.ok || !pg_mt_parse(t, words, p)) return false;
    pos = p;
    return true;
}

} // namespace

const char *pg_game_name(int game_id) { return (game_id >= 0 && game_id < PG_NUM_GAMES) ? NAMES[game_id] : ""; }

std::string pg_mt_text(const uint32_t *words, int pos) {
    std::string t;
    t.reserve(PG_MT_N * 11 + 4);
    for (int i = 0; i < PG_MT_N; i++) {
        t += std::to_string(words[i]);
        t += ' ';
    }
    t += std::to_string(pos);
    return t;
}

bool pg_mt_parse(const std::string &text, uint32_t *words, int &pos) {
    std::istringstream in(text);
    for (int i = 0; i < PG_MT_N; i++) {
        unsigned long long v;
        if (!(in >> v) || v > 0xffffffffull) return false;
        words[i] = (uint32_t)v;
    }
    long p;
    if (!(in >> p) || p < 0 || p > PG_MT_N) return false;
    pos = (int)p;
    return true;
}

void pg_state_write(const HostEnv &h, std::vector<char> &out) {
    const PGEnv &s = h.s;
    const int gid = s.game_id;
    const std::string name = pg_game_name(gid);
    StateWriter w{out};
    // ---- Game::serialize (game.cpp:196-242)
    w.i(SERIALIZE_VERSION);
    w.s(name);
    w.i(s.opt_paint_vel_info); w.i(0 /* use_generated_assets */); w.i(s.opt_use_monochrome_assets);
    w.i(s.opt_restrict_themes); w.i(s.opt_use_backgrounds); w.i(s.opt_center_agent); w.i(s.opt_debug_mode);
    w.i(s.opt_distribution_mode); w.i(s.opt_use_sequential_levels);
    w.i(0); w.i(0); w.i(0); // use_easy_jump, plain_assets, physics_mode (coinrun_old only)
    w.i(s.grid_step); w.i(s.level_seed_low); w.i(s.level_seed_high); w.i(0 /* game_type */); w.i(s.game_n);
    write_randgen(w, h.mt[1], s.lsg_mti);
    write_randgen(w, h.mt[0], s.rg_mti);
    w.f(s.sd_reward); w.i(s.sd_done); w.i(s.sd_level_complete);
    w.i(s.action); w.i(s.timeout);
    w.i(s.current_level_seed); w.i(s.prev_level_seed); w.i(s.episodes_remaining); w.i(s.episode_done);
    w.i(s.last_reward_timer); w.f(s.last_reward); w.i(s.default_action);
    w.i((int32_t)hash_str_uint32(name)); // fixed_asset_seed
    w.i(s.cur_time); w.i(0 /* is_waiting_for_step */);
    // ---- BasicAbstractGame::serialize (basic-abstract-game.cpp:1177-1228)
    w.i(s.main_width * s.main_height); // grid_size
    w.i(s.num_ents);
    for (int k = 0; k < s.num_ents; k++) write_entity(w, h.ent, (size_t)k);
    const ViewM m = view_members(h);
    w.i(0 /* use_procgen_background */); w.i(s.background_index); w.f(s.bg_tile_ratio); w.f(s.bg_pct_x);
    w.f(s.char_dim); w.i(s.last_move_action); w.i(s.move_action); w.i(s.special_action);
    w.f(s.mixrate); w.f(s.maxspeed); w.f(s.max_jump);
    w.f(s.action_vx); w.f(s.action_vy); w.f(s.action_vrot);
    w.f(m.cx); w.f(m.cy);
    w.i(s.random_agent_start); w.i(s.has_useful_vel_info); w.i(s.step_rand_int);
    {
        std::ostringstream o;
        o << std::mt19937(); // asset_rand_gen: never seeded (is_seeded false)
        w.i(0);
        w.s(o.str());
    }
    w.i(s.main_width); w.i(s.main_height); w.i(s.out_of_bounds_object);
    w.f(m.unit); w.f(m.view_dim); w.f(m.x_off); w.f(m.y_off); w.f(m.vis); w.f(s.min_visibility);
    w.i(s.main_width); w.i(s.main_height); // Grid::serialize (grid.h:69-73)
    w.i(s.main_width * s.main_height);
    for (int16_t c : h.cells) w.i(c);
    // ---- the game's serialize
    switch (gid) {
    case PG_GAME_BIGFISH: w.i(s.fish_eaten); w.f(s.r_inc); break;
    case PG_GAME_BOSSFIGHT: {
        const auto &b = s.gs.bf;
        w.i(b.num_rounds);
        for (int i = 0; i < b.num_rounds; i++) w.i((int32_t)((b.attack_modes >> (2 * i)) & 3));
        w.i(s.last_fire_time); w.i(b.time_to_swap); w.i(b.invulnerable_duration); w.i(500 /* vulnerable_duration */);
        w.i(b.num_rounds); w.i(b.round_num); w.i(b.round_health); w.i(20 /* boss_vel_timeout = BOSS_VEL_TIMEOUT */);
        w.i(b.curr_vel_timeout); w.i(b.attack_mode); w.i(b.player_laser_theme); w.i(b.boss_laser_theme);
        w.i(b.damaged_until_time); w.b(b.shields_are_up != 0); w.b(b.barriers_moves_right != 0);
        w.f(0.1f /* base_fire_prob */); w.f(b.boss_bullet_vel); w.f(0.1f /* barrier_vel */);
        w.f(0.025f /* barrier_spawn_prob */); w.f(b.rand_pct); w.f(b.rand_fire_pct); w.f(b.rand_pct_x);
        w.f(b.rand_pct_y);
        break;
    }
    case PG_GAME_CAVEFLYER: break;
    case PG_GAME_CHASER: {
        const int n = s.main_width * s.main_height;
        std::vector<int32_t> free_cells;
        for (int i = 0; i < n; i++)
            if (h.cells[(size_t)i] != 5 /* MAZE_WALL */) free_cells.push_back(i);
        w.i((int32_t)free_cells.size());
        for (int32_t c : free_cells) w.i(c);
        w.i(n);
        for (int i = 0; i < n; i++) w.b(h.cells[(size_t)i] != 5);
        w.i(s.eat_timeout); w.i(s.egg_timeout); w.i(s.eat_time); w.i(s.total_enemies); w.i(s.total_orbs);
        w.i(s.orbs_collected); w.i(s.maze_dim);
        break;
    }
    case PG_GAME_CLIMBER:
        w.b(s.has_support != 0); w.b(s.facing_right != 0); w.i(s.coin_quota); w.i(s.coins_collected);
        w.i(s.wall_theme); w.f(s.gravity); w.f(s.air_control);
        break;
    case PG_GAME_COINRUN:
        w.f(s.last_agent_y); w.i(s.wall_theme); w.b(s.has_support != 0); w.b(s.facing_right != 0);
        w.b(s.is_on_crate != 0); w.f(s.gravity); w.f(s.air_control);
        break;
    case PG_GAME_DODGEBALL:
        w.f(s.db_min_dim); w.f(s.db_hard_min_dim); w.f(s.db_ball_vscale); w.f(s.db_ball_r);
        w.i(s.last_fire_time); w.i(s.num_enemies); w.i(s.enemy_fire_delay);
        break;
    case PG_GAME_FRUITBOT: w.f(5 /* min_dim */); w.f(.5f /* bullet_vscale */); w.i(s.last_fire_time); break;
    case PG_GAME_HEIST:
        w.i(s.num_keys); w.i(s.world_dim); w.i(s.num_keys);
        for (int i = 0; i < s.num_keys; i++) w.b(((s.has_keys >> i) & 1) != 0);
        break;
    case PG_GAME_JUMPER: {
        const auto &j = s.gs.jp;
        w.i(j.jump_count); w.i(j.jump_delta); w.i(j.jump_time); w.b(s.has_support != 0); w.b(s.facing_right != 0);
        w.i(s.wall_theme); w.f(j.compass_dim);
        break;
    }
    case PG_GAME_LEAPER:
        w.i(s.bottom_road_y);
        w.i(s.num_road_lanes);
        for (int i = 0; i < s.num_road_lanes; i++) w.f(s.road_lane_speeds[i]);
        w.i(s.bottom_water_y);
        w.i(s.num_water_lanes);
        for (int i = 0; i < s.num_water_lanes; i++) w.f(s.water_lane_speeds[i]);
        w.i(s.goal_y);
        break;
    case PG_GAME_MAZE: w.i(s.maze_dim); w.i(s.world_dim); break;
    case PG_GAME_MINER: w.i(s.diamonds_remaining); break;
    case PG_GAME_NINJA:
        w.b(s.has_support != 0); w.b(s.facing_right != 0); w.i(s.last_fire_time); w.i(s.wall_theme);
        w.f(s.gravity); w.f(s.air_control); w.f(s.gs.nj.jump_charge); w.f(s.gs.nj.jump_charge_inc);
        break;
    case PG_GAME_PLUNDER: {
        const auto &p = s.gs.pl;
        w.i(s.last_fire_time);
        w.i(p.num_lanes);
        for (int i = 0; i < p.num_lanes; i++) w.b(((p.lane_dirs >> i) & 1) != 0);
        w.i(6); // num_total_ship_types (plunder.cpp:127)
        for (int i = 0; i < 6; i++) w.b(((p.target_bools >> i) & 1) != 0);
        w.i(6);
        for (int i = 0; i < 6; i++) w.i((int32_t)((p.perm >> (4 * i)) & 15));
        w.i(p.num_lanes);
        for (int i = 0; i < p.num_lanes; i++) w.f(p.lane_vels[i]);
        w.i(p.num_lanes); w.i(p.num_current_ship_types); w.i(p.targets_hit); w.i(p.target_quota);
        w.f(p.juice_left); w.f(p.r_scale); w.f(p.spawn_prob); w.f(p.legend_r); w.f(p.min_agent_x);
        break;
    }
    case PG_GAME_STARPILOT: // write_entities(b, spawners): spawners[i] = slot PG_CAP - 1 - i
        w.i(s.num_tail);
        for (int i = 0; i < s.num_tail; i++) write_entity(w, h.tail, (size_t)(s.num_tail - 1 - i));
        break;
    default: break;
    }
    w.i(END_OF_BUFFER);
}

bool pg_state_read(const char *data, size_t length, HostEnv &h, std::string &err) {
    StateReader r{data, length, 0, true};
    PGEnv s = h.s;
    const int gid = s.game_id;
    auto bad = [&](const char *msg) {
        err = msg;
        return false;
    };
    // ---- Game::deserialize (game.cpp:257-304)
    if (r.i() != SERIALIZE_VERSION) return bad("set_state: SERIALIZE_VERSION mismatch");
    if (r.s() != pg_game_name(gid)) return bad("set_state: the state belongs to another game than this env slot");
    s.opt_paint_vel_info = r.i();
    if (r.i()) return bad("set_state: use_generated_assets states are not supported (basic-abstract-game.cpp:1183)");
    s.opt_use_monochrome_assets = r.i(); s.opt_restrict_themes = r.i(); s.opt_use_backgrounds = r.i();
    s.opt_center_agent = r.i(); s.opt_debug_mode = r.i(); s.opt_distribution_mode = r.i();
    s.opt_use_sequential_levels = r.i();
    if (r.i() || r.i() || r.i()) return bad("set_state: coinrun_old options are not supported");
    s.grid_step = r.i(); s.level_seed_low = r.i(); s.level_seed_high = r.i();
    r.i(); // game_type
    s.game_n = r.i();
    if (!read_randgen(r, h.mt[1], s.lsg_mti) || !read_randgen(r, h.mt[0], s.rg_mti))
        return bad("set_state: bad RandGen state");
    s.sd_reward = r.f(); s.sd_done = r.i(); s.sd_level_complete = r.i();
    s.action = r.i(); s.timeout = r.i();
    s.current_level_seed = r.i(); s.prev_level_seed = r.i(); s.episodes_remaining = r.i(); s.episode_done = r.i();
    s.last_reward_timer = r.i(); s.last_reward = r.f(); s.default_action = r.i();
    r.i(); // fixed_asset_seed: used by generated assets only
    s.cur_time = r.i();
    r.i(); // is_waiting_for_step
    // ---- BasicAbstractGame::deserialize (basic-abstract-game.cpp:1230-1280)
    const int grid_size = r.i();
    const int ne = r.count(PG_CAP);
    std::vector<int32_t> ent[PG_NF];
    for (int f = 0; f < PG_NF; f++) ent[f].assign((size_t)ne, 0);
    for (int k = 0; k < ne && r.ok; k++) read_entity(r, ent, (size_t)k);
    if (!r.ok) return bad("set_state: truncated entity list");
    // fassert(agent_idx >= 0) (:1238-1240); this engine keeps the agent in slot 0, where every
    // reset puts it and order-preserving erase keeps it
    if (ne == 0 || ent[F_TYPE][0] != 0) return bad("set_state: entity 0 is not the agent (PLAYER)");
    if (r.i()) return bad("set_state: procedurally generated backgrounds are not supported");
    s.background_index = r.i(); s.bg_tile_ratio = r.f(); s.bg_pct_x = r.f();
    s.char_dim = r.f(); s.last_move_action = r.i(); s.move_action = r.i(); s.special_action = r.i();
    s.mixrate = r.f(); s.maxspeed = r.f(); s.max_jump = r.f();
    s.action_vx = r.f(); s.action_vy = r.f(); s.action_vrot = r.f();
    r.f(); r.f(); // center_x, center_y: recomputed by every render
    s.random_agent_start = r.i(); s.has_useful_vel_info = r.i(); s.step_rand_int = r.i();
    r.i(); r.s(); // asset_rand_gen
    s.main_width = r.i(); s.main_height = r.i(); s.out_of_bounds_object = r.i();
    r.f(); r.f(); r.f(); r.f(); // unit, view_dim, x_off, y_off
    const float vis = r.f();
    s.min_visibility = r.f();
    // the render uses the member visibility as is only for centred views of games without their
    // own choose_center; every other frame recomputes it (prepare_for_drawing)
    if (s.opt_center_agent && gid != PG_GAME_CLIMBER && gid != PG_GAME_FRUITBOT) s.visibility = vis;
    const int gw = r.i(), gh = r.i();
    const int nc = r.count(PG_GRID_MAX);
    if (!r.ok || gw != s.main_width || gh != s.main_height || nc != gw * gh || grid_size != nc || gw <= 0 || gh <= 0)
        return bad("set_state: grid dimensions do not match the world");
    std::vector<int16_t> cells((size_t)nc);
    for (int k = 0; k < nc; k++) {
        const int32_t c = r.i();
        if (c < -32768 || c > 32767) return bad("set_state: grid value out of range");
        cells[(size_t)k] = (int16_t)c;
    }
    std::vector<int32_t> tl[PG_NF];
    int num_tail = 0;
    // ---- the game's deserialize
    switch (gid) {
    case PG_GAME_BIGFISH: s.fish_eaten = r.i(); s.r_inc = r.f(); break;
    case PG_GAME_BOSSFIGHT: {
        auto &b = s.gs.bf;
        const int nm = r.count(5);
        uint32_t am = 0;
        for (int i = 0; i < nm; i++) am |= (uint32_t)(r.i() & 3) << (2 * i);
        b.attack_modes = am;
        s.last_fire_time = r.i(); b.time_to_swap = r.i(); b.invulnerable_duration = r.i();
        if (r.i() != 500) return bad("set_state: bossfight vulnerable_duration differs from the game's constant");
        b.num_rounds = r.i(); b.round_num = r.i(); b.round_health = r.i();
        if (r.i() != 20) return bad("set_state: bossfight boss_vel_timeout differs from the game's constant");
        b.curr_vel_timeout = r.i(); b.attack_mode = r.i(); b.player_laser_theme = r.i(); b.boss_laser_theme = r.i();
        b.damaged_until_time = r.i(); b.shields_are_up = r.b(); b.barriers_moves_right = r.b();
        if (r.f() != 0.1f) return bad("set_state: bossfight base_fire_prob differs from the game's constant");
        b.boss_bullet_vel = r.f();
        if (r.f() != 0.1f || r.f() != 0.025f) return bad("set_state: bossfight barrier constants differ");
        b.rand_pct = r.f(); b.rand_fire_pct = r.f(); b.rand_pct_x = r.f(); b.rand_pct_y = r.f();
        if (nm != b.num_rounds) return bad("set_state: bossfight attack_modes size != num_rounds");
        break;
    }
    case PG_GAME_CAVEFLYER: break;
    case PG_GAME_CHASER: {
        const int nf = r.count(PG_GRID_MAX);
        for (int i = 0; i < nf; i++) r.i(); // free_cells: derived from the grid
        const int ns = r.count(PG_GRID_MAX);
        for (int i = 0; i < ns; i++) r.i(); // is_space_vec: derived from the grid
        s.eat_timeout = r.i(); s.egg_timeout = r.i(); s.eat_time = r.i(); s.total_enemies = r.i();
        s.total_orbs = r.i(); s.orbs_collected = r.i(); s.maze_dim = r.i();
        break;
    }
    case PG_GAME_CLIMBER:
        s.has_support = r.b(); s.facing_right = r.b(); s.coin_quota = r.i(); s.coins_collected = r.i();
        s.wall_theme = r.i(); s.gravity = r.f(); s.air_control = r.f();
        break;
    case PG_GAME_COINRUN:
        s.last_agent_y = r.f(); s.wall_theme = r.i(); s.has_support = r.b(); s.facing_right = r.b();
        s.is_on_crate = r.b(); s.gravity = r.f(); s.air_control = r.f();
        break;
    case PG_GAME_DODGEBALL:
        s.db_min_dim = r.f(); s.db_hard_min_dim = r.f(); s.db_ball_vscale = r.f(); s.db_ball_r = r.f();
        s.last_fire_time = r.i(); s.num_enemies = r.i(); s.enemy_fire_delay = r.i();
        break;
    case PG_GAME_FRUITBOT:
        if (r.f() != 5 || r.f() != .5f) return bad("set_state: fruitbot constants differ");
        s.last_fire_time = r.i();
        break;
    case PG_GAME_HEIST: {
        s.num_keys = r.i(); s.world_dim = r.i();
        const int nk = r.count(31);
        int32_t hk = 0;
        for (int i = 0; i < nk; i++)
            if (r.b()) hk |= 1 << i;
        s.has_keys = hk;
        if (nk != s.num_keys) return bad("set_state: heist has_keys size != num_keys");
        break;
    }
    case PG_GAME_JUMPER: {
        auto &j = s.gs.jp;
        j.jump_count = r.i(); j.jump_delta = r.i(); j.jump_time = r.i(); s.has_support = r.b(); s.facing_right = r.b();
        s.wall_theme = r.i(); j.compass_dim = r.f();
        break;
    }
    case PG_GAME_LEAPER: {
        s.bottom_road_y = r.i();
        s.num_road_lanes = r.count(5);
        for (int i = 0; i < s.num_road_lanes; i++) s.road_lane_speeds[i] = r.f();
        s.bottom_water_y = r.i();
        s.num_water_lanes = r.count(5);
        for (int i = 0; i < s.num_water_lanes; i++) s.water_lane_speeds[i] = r.f();
        s.goal_y = r.i();
        break;
    }
    case PG_GAME_MAZE: s.maze_dim = r.i(); s.world_dim = r.i(); break;
    case PG_GAME_MINER: s.diamonds_remaining = r.i(); break;
    case PG_GAME_NINJA:
        s.has_support = r.b(); s.facing_right = r.b(); s.last_fire_time = r.i(); s.wall_theme = r.i();
        s.gravity = r.f(); s.air_control = r.f(); s.gs.nj.jump_charge = r.f(); s.gs.nj.jump_charge_inc = r.f();
        break;
    case PG_GAME_PLUNDER: {
        auto &p = s.gs.pl;
        s.last_fire_time = r.i();
        const int nd = r.count(5);
        uint32_t dirs = 0;
        for (int i = 0; i < nd; i++)
            if (r.b()) dirs |= 1u << i;
        const int nt = r.count(6);
        uint32_t tb = 0;
        for (int i = 0; i < nt; i++)
            if (r.b()) tb |= 1u << i;
        const int np = r.count(6);
        uint32_t perm = 0;
        for (int i = 0; i < np; i++) perm |= (uint32_t)(r.i() & 15) << (4 * i);
        const int nv = r.count(5);
        float vels[5] = {0, 0, 0, 0, 0};
        for (int i = 0; i < nv; i++) vels[i] = r.f();
        p.lane_dirs = dirs; p.target_bools = tb; p.perm = perm;
        for (int i = 0; i < 5; i++) p.lane_vels[i] = vels[i];
        p.num_lanes = r.i(); p.num_current_ship_types = r.i(); p.targets_hit = r.i(); p.target_quota = r.i();
        p.juice_left = r.f(); p.r_scale = r.f(); p.spawn_prob = r.f(); p.legend_r = r.f(); p.min_agent_x = r.f();
        if (nd != p.num_lanes || nv != p.num_lanes || nt != 6 || np != 6)
            return bad("set_state: plunder vector sizes do not match");
        break;
    }
    case PG_GAME_STARPILOT: {
        num_tail = r.count(PG_CAP);
        for (int f = 0; f < PG_NF; f++) tl[f].assign((size_t)num_tail, 0);
        std::vector<int32_t> sp[PG_NF];
        for (int f = 0; f < PG_NF; f++) sp[f].assign((size_t)num_tail, 0);
        for (int i = 0; i < num_tail && r.ok; i++) read_entity(r, sp, (size_t)i);
        for (int i = 0; i < num_tail; i++) // spawners[i] -> tail index num_tail - 1 - i
            for (int f = 0; f < PG_NF; f++) tl[f][(size_t)(num_tail - 1 - i)] = sp[f][(size_t)i];
        break;
    }
    default: break;
    }
    if (!r.ok) return bad("set_state: truncated state");
    if (r.i() != END_OF_BUFFER || !r.ok) return bad("set_state: missing END_OF_BUFFER");
    if (ne + num_tail > PG_CAP) return bad("set_state: more entities than this build's slots");
    s.num_ents = ne;
    s.num_tail = num_tail;
    s.agent_erased = 0;
    s.grid8_ok = 0; // the int8 mirror is rebuilt at the next reset; until then the step reads int16
    s.error = 0;
    h.s = s;
    for (int f = 0; f < PG_NF; f++) {
        h.ent[f] = ent[f];
        if (gid == PG_GAME_STARPILOT) h.tail[f] = tl[f];
    }
    if (gid != PG_GAME_STARPILOT)
        for (int f = 0; f < PG_NF; f++) h.tail[f].clear(), h.s.num_tail = 0;
    h.cells = cells;
    return true;
}
