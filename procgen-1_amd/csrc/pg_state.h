// pg_state.h -- one env's state on the host, and the upstream get_state / set_state byte format.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "pg_engine.h"

// One env copied out of HBM: the PGEnv block, the live entity planes (slots 0..ents-1), the
// reserved top slots (starpilot's spawners, slot PG_CAP - 1 - i = spawners[i]), the grid and both
// generators ([0] rand_gen, [1] level_seed_rand_gen: 624 words, the position is in PGEnv).
struct HostEnv {
    PGEnv s;
    std::vector<int32_t> ent[PG_NF];  // [field][slot], ents = s.num_ents
    std::vector<int32_t> tail[PG_NF]; // [field][k], slot PG_CAP - s.num_tail + k
    std::vector<int16_t> cells;       // main_width * main_height
    uint32_t mt[2][PG_MT_WORDS];
};

const char *pg_game_name(int game_id);

// Game::serialize + BasicAbstractGame::serialize + the game's serialize (reference game.cpp:196-256,
// basic-abstract-game.cpp:1177-1228, games/*.cpp) with buffer.h's 4-byte writes, then END_OF_BUFFER
// (vecgame.cpp:6, 486-493).
void pg_state_write(const HostEnv &h, std::vector<char> &out);

// The matching deserialize into `h` (which holds the slot's current state: fields the format does
// not carry keep their values).  False with a message when the bytes are not a state of this
// slot's game that this build can run.
bool pg_state_read(const char *data, size_t length, HostEnv &h, std::string &err);

// RandGen::serialize's text of a std::mt19937 (libstdc++ operator<<: the 624 words, then the position)
std::string pg_mt_text(const uint32_t *words, int pos);
bool pg_mt_parse(const std::string &text, uint32_t *words, int &pos);
