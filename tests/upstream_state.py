"""Reader of the upstream get_state byte format, written from the reference's serialize functions
(game.cpp:196-256, basic-abstract-game.cpp:1177-1228, entity.cpp:90-134, grid.h:69-73, the
games' serialize overrides; buffer.h with its 4-byte writes) for the tests: it walks one state and
returns the fields by name, so a test can check them against the oracle and that the bytes end
exactly at END_OF_BUFFER (vecgame.cpp:6)."""
import struct

END_OF_BUFFER = 0xCAFECAFE
ENTITY = (["x", "y", "vx", "vy", "rx", "ry"], ["type", "image_type", "image_theme", "render_z", "will_erase",
                                                "collides_with_entities"],
          ["collision_margin", "rotation", "vrot"],
          ["is_reflected", "fire_time", "spawn_time", "life_time", "expire_time", "use_abs_coords"], ["friction"],
          ["smart_step", "avoids_collisions", "auto_erase"],
          ["alpha", "health", "theta", "grow_rate", "alpha_decay", "climber_spawn_x"])
GAME_FIELDS = {  # (kind, name): i int, f float, b bool, vi / vb / vf vectors, ents entity list
    "bigfish": [("i", "fish_eaten"), ("f", "r_inc")],
    "bossfight": [("vi", "attack_modes")] + [("i", n) for n in (
        "last_fire_time", "time_to_swap", "invulnerable_duration", "vulnerable_duration", "num_rounds", "round_num",
        "round_health", "boss_vel_timeout", "curr_vel_timeout", "attack_mode", "player_laser_theme",
        "boss_laser_theme", "damaged_until_time")] + [("b", "shields_are_up"), ("b", "barriers_moves_right")] + [
        ("f", n) for n in ("base_fire_prob", "boss_bullet_vel", "barrier_vel", "barrier_spawn_prob", "rand_pct",
                           "rand_fire_pct", "rand_pct_x", "rand_pct_y")],
    "caveflyer": [],
    "chaser": [("vi", "free_cells"), ("vb", "is_space_vec")] + [("i", n) for n in (
        "eat_timeout", "egg_timeout", "eat_time", "total_enemies", "total_orbs", "orbs_collected", "maze_dim")],
    "climber": [("b", "has_support"), ("b", "facing_right"), ("i", "coin_quota"), ("i", "coins_collected"),
                ("i", "wall_theme"), ("f", "gravity"), ("f", "air_control")],
    "coinrun": [("f", "last_agent_y"), ("i", "wall_theme"), ("b", "has_support"), ("b", "facing_right"),
                ("b", "is_on_crate"), ("f", "gravity"), ("f", "air_control")],
    "dodgeball": [("f", "min_dim"), ("f", "hard_min_dim"), ("f", "ball_vscale"), ("f", "ball_r"),
                  ("i", "last_fire_time"), ("i", "num_enemies"), ("i", "enemy_fire_delay")],
    "fruitbot": [("f", "min_dim"), ("f", "bullet_vscale"), ("i", "last_fire_time")],
    "heist": [("i", "num_keys"), ("i", "world_dim"), ("vb", "has_keys")],
    "jumper": [("i", "jump_count"), ("i", "jump_delta"), ("i", "jump_time"), ("b", "has_support"),
               ("b", "facing_right"), ("i", "wall_theme"), ("f", "compass_dim")],
    "leaper": [("i", "bottom_road_y"), ("vf", "road_lane_speeds"), ("i", "bottom_water_y"),
               ("vf", "water_lane_speeds"), ("i", "goal_y")],
    "maze": [("i", "maze_dim"), ("i", "world_dim")],
    "miner": [("i", "diamonds_remaining")],
    "ninja": [("b", "has_support"), ("b", "facing_right"), ("i", "last_fire_time"), ("i", "wall_theme"),
              ("f", "gravity"), ("f", "air_control"), ("f", "jump_charge"), ("f", "jump_charge_inc")],
    "plunder": [("i", "last_fire_time"), ("vb", "lane_directions"), ("vb", "target_bools"),
                ("vi", "image_permutation"), ("vf", "lane_vels")] + [("i", n) for n in (
                    "num_lanes", "num_current_ship_types", "targets_hit", "target_quota")] + [
        ("f", n) for n in ("juice_left", "r_scale", "spawn_prob", "legend_r", "min_agent_x")],
    "starpilot": [("ents", "spawners")],
}


class _R:
    def __init__(self, b):
        self.b, self.o = b, 0

    def i(self):
        v = struct.unpack_from("<i", self.b, self.o)[0]
        self.o += 4
        return v

    def f(self):
        v = struct.unpack_from("<f", self.b, self.o)[0]
        self.o += 4
        return v

    def s(self):
        n = self.i()
        v = bytes(self.b[self.o:self.o + n])
        self.o += n
        return v

    def ent(self):
        e = {}
        for names, fl in zip(ENTITY, (True, False, True, False, True, False, True)):
            for n in names:
                e[n] = self.f() if fl else self.i()
        return e

    def ents(self):
        return [self.ent() for _ in range(self.i())]


def entity_words(e):
    """One parsed entity as the 31 int32 words it was written as (floats as their bits)."""
    out = []
    for names, fl in zip(ENTITY, (True, False, True, False, True, False, True)):
        for n in names:
            out.append(struct.unpack("<i", struct.pack("<f", e[n]))[0] if fl else int(e[n]))
    return out


def randgen(r):
    seeded = r.i()
    words = r.s().split()
    return dict(is_seeded=seeded, words=[int(w) for w in words[:-1]], pos=int(words[-1]))


def parse(b, game):
    r = _R(b)
    d = {"version": r.i(), "game_name": r.s().decode()}
    for n in ("paint_vel_info", "use_generated_assets", "use_monochrome_assets", "restrict_themes", "use_backgrounds",
              "center_agent", "debug_mode", "distribution_mode", "use_sequential_levels", "use_easy_jump",
              "plain_assets", "physics_mode", "grid_step", "level_seed_low", "level_seed_high", "game_type", "game_n"):
        d[n] = r.i()
    d["level_seed_rand_gen"] = randgen(r)
    d["rand_gen"] = randgen(r)
    d["reward"] = r.f()
    for n in ("done", "level_complete", "action", "timeout", "current_level_seed", "prev_level_seed",
              "episodes_remaining", "episode_done", "last_reward_timer"):
        d[n] = r.i()
    d["last_reward"] = r.f()
    for n in ("default_action", "fixed_asset_seed", "cur_time", "is_waiting_for_step", "grid_size"):
        d[n] = r.i()
    d["entities"] = r.ents()
    d["use_procgen_background"], d["background_index"] = r.i(), r.i()
    d["bg_tile_ratio"], d["bg_pct_x"], d["char_dim"] = r.f(), r.f(), r.f()
    d["last_move_action"], d["move_action"], d["special_action"] = r.i(), r.i(), r.i()
    for n in ("mixrate", "maxspeed", "max_jump", "action_vx", "action_vy", "action_vrot", "center_x", "center_y"):
        d[n] = r.f()
    for n in ("random_agent_start", "has_useful_vel_info", "step_rand_int"):
        d[n] = r.i()
    d["asset_rand_gen"] = randgen(r)
    for n in ("main_width", "main_height", "out_of_bounds_object"):
        d[n] = r.i()
    for n in ("unit", "view_dim", "x_off", "y_off", "visibility", "min_visibility"):
        d[n] = r.f()
    gw, gh, gn = r.i(), r.i(), r.i()
    d["grid"] = dict(w=gw, h=gh, data=[r.i() for _ in range(gn)])
    for kind, name in GAME_FIELDS[game]:
        if kind == "i":
            d[name] = r.i()
        elif kind == "f":
            d[name] = r.f()
        elif kind == "b":
            d[name] = bool(r.i())
        elif kind == "ents":
            d[name] = r.ents()
        else:
            n = r.i()
            d[name] = [r.f() if kind == "vf" else (bool(r.i()) if kind == "vb" else r.i()) for _ in range(n)]
    d["end"] = r.i() & 0xffffffff
    d["consumed"] = r.o
    return d
