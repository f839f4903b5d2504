// Tile configurations and LDS geometry of the K-streamed tile kernel (conv_tile.hip).
#pragma once
#include "conv_common.h"

namespace sddm {

// tile configurations: waves along pixels, waves along output channels, 16-pixel fragments per
// wave, 16-channel fragments per wave, staging units per thread and chunk (stride 1 / stride 2)
struct TileCfgX { int wpx, wco, fp, fc, maxu, maxu_s2; };
static constexpr TileCfgX kTileCfgs[] = {
    {4, 2, 4, 2, 4, 10},   //  0: 256 px x 64 co, 8 waves
    {8, 1, 2, 2, 4, 10},   //  1: 256 px x 32 co, 8 waves
    {4, 2, 2, 2, 3, 6},    //  2: 128 px x 64 co, 8 waves
    {4, 2, 4, 3, 4, 10},   //  3: 256 px x 96 co, 8 waves
    {4, 1, 2, 2, 5, 11},   //  4: 128 px x 32 co, 4 waves
    {2, 2, 2, 2, 4, 8},    //  5:  64 px x 64 co, 4 waves
    {2, 4, 2, 1, 2, 5},    //  6:  64 px x 64 co, 8 waves
    {1, 4, 2, 1, 2, 5},    //  7:  32 px x 64 co, 4 waves
    {1, 2, 2, 1, 2, 5},    //  8:  32 px x 32 co, 2 waves
    {1, 1, 2, 1, 4, 10},   //  9:  32 px x 16 co, 1 wave
    {4, 2, 2, 3, 3, 6},    // 10: 128 px x 96 co, 8 waves
    {2, 1, 2, 2, 4, 10},   // 11:  64 px x 32 co, 2 waves
    {8, 1, 4, 2, 6, 10},   // 12: 512 px x 32 co, 8 waves (the 128 x 64 level in one round of blocks; stride 1)
};
static constexpr int kNTileCfgs = (int)(sizeof(kTileCfgs) / sizeof(kTileCfgs[0]));

struct TileGeo { int HR, HC, HE, HP, PLB, nu3, nur, ibb; };

__host__ __device__ inline TileGeo tile_geo(bool s2, int TR, int TW, int MT, bool res) {
  TileGeo g;
  g.HR = s2 ? 2 * TR + 1 : TR + 2;
  g.HC = s2 ? 2 * TW + 1 : TW + 2;
  g.HE = (g.HC + 1) / 2;                                  // even halo columns (stride 2)
  g.HP = g.HR * g.HC;
  const int slots = g.HP > MT ? g.HP : MT;
  g.PLB = (slots * 16 + 255) / 256 * 256;                 // plane bytes (the swizzle stays inside)
  g.nu3 = g.HP * 4;                                       // 16-byte units of one 32-channel chunk
  g.nur = res ? MT * 4 : 0;
  g.ibb = 4 * g.PLB;
  return g;
}

// LDS: two operand images, two weight chunks (576 B per output channel), GroupNorm scale / shift;
// a single K chunk (nk == 1) needs one of each
__host__ __device__ inline int tile_lds(const TileGeo& g, int NB, int Cin, int nbuf) {
  return nbuf * g.ibb + nbuf * 576 * NB + 2 * Cin * 4;
}

__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

}  // namespace sddm
