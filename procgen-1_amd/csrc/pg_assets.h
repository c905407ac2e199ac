// pg_assets.h -- host-side asset loader: builds the engine's sprite atlas inside libenv_make.
//
// Reference: VecGame's first construction runs global_init -> images_load (vecgame.cpp:144-153,
// 189-193; resources.cpp:20-30, 837-979), which decodes every PNG under resource_root and each
// game then picks its images (asset_for_type, basic-abstract-game.cpp:93-121).  This build ships
// the images Qt-decoded into compressed .npz packs plus a manifest of every game's tables
// (procgen-1_amd/assets/, tools/make_asset_manifest.py); pg_atlas_load reads them (zip + deflate
// via zlib, .npy headers parsed here) and lays out one pixel array for the games of a batch,
// each distinct image once.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

struct PGAtlasHost {
    std::vector<uint32_t> pixels;          // 0xAARRGGBB
    std::vector<int32_t> sprites;          // [16][1000][4] offset, w, h, 0
    std::vector<int32_t> backgrounds;      // [16][64][4]
    std::vector<int32_t> num_backgrounds;  // [16]
    std::vector<int32_t> num_themes;       // [16][100]
};

// Default asset directory: <directory of this shared library>/../assets.
std::string pg_default_asset_root();

// Build the atlas of the given game ids from `root` (a directory holding manifest.txt and the
// packs).  Returns false with `err` set when a file is missing or malformed.
bool pg_atlas_load(const std::string &root, const std::vector<int> &games, PGAtlasHost *out, std::string *err);
