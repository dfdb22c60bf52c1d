p='/root/repo/raytracer-cuda_amd/csrc/crt_hip.hip'; s=open(p).read()
def rep(old, new, cnt=1):
    global s
    assert s.count(old) == cnt, (old[:80], s.count(old))
    s = s.replace(old, new)
# params
rep('''    int crit_tiles, crit_threshold;       // variant 8: the first crit_tiles tiles of the cost order regenerate at
                                          // crit_threshold parked lanes instead of regen_threshold
};''','''    int crit_tiles, crit_threshold;       // variant 8: the first crit_tiles tiles of the cost order regenerate at
                                          // crit_threshold parked lanes instead of regen_threshold
    int refill_below;                     // variant 7: lanes without a pixel take new ones only while fewer than this
                                          // many lanes of the wave hold a pixel (64: always)
};''')
# kernel: refill only when the wave has fewer than refill_below pixels
rep('''                while (!exhausted) {                // lanes without a pixel take the next slots''','''                // lanes without a pixel take the next slots: always (refill_below 64), or only once fewer than
                // refill_below lanes of the wave still hold a pixel, so a wave keeps its first tile until it drains
                const bool refill = __popcll(wave_ballot(have)) < P.refill_below;
                while (refill && !exhausted) {''')
# tile expansion kernel generalised with an optional tile order
rep('''__global__ void crt_order_tiles_kernel(uint32_t* __restrict__ order, int width, int height, int n_slots) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    const int tiles_x = (width + 7) / 8, tile = s >> 6, q = s & 63;''','''__global__ void crt_order_tiles_kernel(uint32_t* __restrict__ order, int width, int height, int n_slots,
                                       const uint32_t* __restrict__ tile_order = nullptr) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    const int tiles_x = (width + 7) / 8, tile = tile_order ? (int)tile_order[s >> 6] : s >> 6, q = s & 63;''')
# renderer state
rep('''    uint32_t* d_tile_key = nullptr;    // variant 8: per-tile keys''','''    uint32_t* d_tile_key = nullptr;    // variant 8: per-tile keys
    uint32_t* d_tile_order = nullptr;  // variant 7 with refill_below < 64: tiles most expensive first
    int refill_below = 64;             // variant 7: see RenderParams::refill_below''')
rep('''    if (R->d_tile_key) (void)hipFree(R->d_tile_key);''','''    if (R->d_tile_key) (void)hipFree(R->d_tile_key);
    if (R->d_tile_order) (void)hipFree(R->d_tile_order);''')
rep('''    P.order = nullptr; P.queue = nullptr; P.n_slots = 0; P.probe_cost = nullptr; P.tiles_x = 0; P.crit_tiles = 0; P.crit_threshold = 64;''',
'''    P.order = nullptr; P.queue = nullptr; P.n_slots = 0; P.probe_cost = nullptr; P.tiles_x = 0; P.crit_tiles = 0; P.crit_threshold = 64;
    P.refill_below = R->refill_below;''')
# host: variant 7 with refill_below < 64 and a probe: tile-cost order expanded to pixel slots
rep('''        if (probe_spp_for(R, spp) > 0) {
            // cost probe: variant 4 at probe_spp samples over the same RNG state, read-only: rays per pixel''','''        if (probe_spp_for(R, spp) > 0 && R->refill_below < 64) {
            // tiles most expensive first (variant 8's probe, tile keys and sort), each tile's 64 pixels consecutive:
            // a wave's first 64 slots are one tile, and it refills from the next tiles once it has drained
            const int n_tiles = tiles_x * tiles_y;
            if (!R->d_tile_order) {
                HIP_TRY(hipStreamSynchronize(st));
                HIP_TRY(hipMalloc((void**)&R->d_tile_order, (size_t)n_tiles * 4));
                if (!R->d_tile_key) HIP_TRY(hipMalloc((void**)&R->d_tile_key, (size_t)n_tiles * 4));
            }
            RenderParams Q = P;
            Q.spp = probe_spp_for(R, spp);
            Q.accumulate = 0;
            Q.probe_cost = R->d_tile_cost;
            if (occ >= 6) hipLaunchKernelGGL((crt_render_kernel<true, 4, 6>), grid, block, 0, st, Q);
            else hipLaunchKernelGGL((crt_render_kernel<true, 4, 5>), grid, block, 0, st, Q);
            hipLaunchKernelGGL(crt_tile_cost_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, st, R->d_tile_cost,
                               R->width, R->height, tiles_x, n_tiles, R->d_tile_key, R->tile_key_mode);
            if (R->tile_key_mode == 2) {
                hipLaunchKernelGGL(crt_tile_neighbour_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, st,
                                   R->d_tile_key, tiles_x, n_tiles, R->d_tile_cost);
                HIP_TRY(hipMemcpyAsync(R->d_tile_key, R->d_tile_cost, (size_t)n_tiles * 4, hipMemcpyDeviceToDevice, st));
            }
            const unsigned ob = (unsigned)((n_tiles + ORDER_ITEMS - 1) / ORDER_ITEMS);
            HIP_TRY(hipMemsetAsync(R->d_order_hist, 0, ORDER_KEYS * 4, st));
            hipLaunchKernelGGL(crt_order_hist_kernel, dim3(ob), dim3(256), 0, st, R->d_tile_key, n_tiles, R->d_order_hist);
            hipLaunchKernelGGL(crt_order_scan_kernel, dim3(1), dim3(ORDER_KEYS), 0, st, R->d_order_hist);
            hipLaunchKernelGGL(crt_order_scatter_kernel, dim3(ob), dim3(256), 0, st, R->d_tile_key, n_tiles,
                               R->d_order_hist, R->d_tile_order, 0u);
            hipLaunchKernelGGL(crt_order_tiles_kernel, dim3((unsigned)((n_tile_slots + 255) / 256)), dim3(256), 0, st,
                               R->d_order, R->width, R->height, (int)n_tile_slots, (const uint32_t*)R->d_tile_order);
            P.n_slots = (int)n_tile_slots;
        } else if (probe_spp_for(R, spp) > 0) {
            // cost probe: variant 4 at probe_spp samples over the same RNG state, read-only: rays per pixel''')
rep('''int crt_renderer_set_critical_tiles(crt_renderer* R, int tiles, int lanes) {''','''int crt_renderer_set_refill(crt_renderer* R, int below) {
    if (!R || below < 1 || below > 64) return set_error(CRT_ERR_INVALID_ARGUMENT, "refill threshold 1..64");
    R->refill_below = below;
    return CRT_OK;
}

int crt_renderer_set_critical_tiles(crt_renderer* R, int tiles, int lanes) {''')
open(p,'w').write(s)
p='/root/repo/include/crt_hip.h'; s=open(p).read()
old='''int  crt_renderer_set_critical_tiles(crt_renderer* r, int tiles, int lanes);'''
assert old in s
s=s.replace(old, old+'''
/* Variant 7 (persistent waves, lanes take pixels from a queue): lanes without a pixel take new ones only while fewer
 * than `below` lanes of the wave hold a pixel (1..64; 64 = always, the default).  Below 64 and with the cost probe,
 * the queue holds whole 8x8 tiles most expensive first, so a wave starts with one tile and tops up from the next
 * tiles once it has drained below `below` pixels.  Same frames for every value. */
int  crt_renderer_set_refill(crt_renderer* r, int below);''')
open(p,'w').write(s)
p='/root/repo/raytracer-cuda_amd/crt_amd/_lib.py'; s=open(p).read()
s=s.replace('''"crt_renderer_set_schedule", "crt_renderer_set_critical_tiles",''','''"crt_renderer_set_schedule", "crt_renderer_set_critical_tiles", "crt_renderer_set_refill",''',1)
old='''            "crt_renderer_synchronize": ([P, P], i32),'''
assert old in s
s=s.replace(old, '''            "crt_renderer_set_refill": ([P, i32], i32),
'''+old,1)
open(p,'w').write(s)
p='/root/repo/raytracer-cuda_amd/crt_amd/__init__.py'; s=open(p).read()
old='''    def set_kernel_variant(self, variant: int):'''
assert old in s
s=s.replace(old,'''    def set_refill(self, below: int = 64):
        check(_lib.hip().crt_renderer_set_refill(self.h, int(below)), "set_refill")

'''+old,1)
open(p,'w').write(s)
print("patched")
