// Host-side check of the fused-MLP layout plan (robust-nerf_amd/csrc/mlp_plan.cpp.inc):
// every parameter's gradient is read by the dW reduction from a slab entry that
// exactly one dW wave share writes, and every share stays inside its job's grid.
//   plan_check pos_freqs dir_freqs n_layers skip_mask use_view_dirs precision
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <set>
#include <tuple>
#include "mlp_plan.hpp"
namespace nr {
static int ceil_div(int a, int b) { return (a + b - 1) / b; }
}
#include "mlp_plan.cpp.inc"
using namespace nr;
int main(int argc, char** argv) {
    NrMlpConfig c{10, 4, 256, 8, 1u << 4, 1, 1};
    if (argc == 7) c = {atoi(argv[1]), atoi(argv[2]), 256, atoi(argv[3]), (uint32_t)atoi(argv[4]), atoi(argv[5]), atoi(argv[6])};
    MlpPlan p; const char* why = "";
    if (!make_plan(&c, &p, &why)) { printf("plan fail %s\n", why); return 1; }
    std::set<std::tuple<int,int,int>> written;  // job,row,col
    long dup = 0;
    for (int j = 0; j < p.n_jobs; ++j) {
        const DwJob& jb = p.job[j];
        printf("job %d NBz %d KB %d waves %d:", j, jb.NBz, jb.KB, jb.nwaves);
        // the dW kernel stages at most dw_max_pieces 1-KB pieces per wave and tile
        if ((jb.NBz + jb.KB) * p.fpb > kDwMaxWaves * dw_max_pieces(p.fpb == 2)) {
            printf("\nstaging exceeds the per-wave pieces\n");
            return 1;
        }
        for (int v = 0; v < jb.nwaves; ++v) {
            const DwWave& w = jb.w[v];
            printf(" [%d+%d x %d+%d%s]", w.row0, w.np, w.col0, w.nq, w.bias ? " b" : "");
            if (w.np < 1 || w.np > kDwMaxP || w.nq < 1 || w.nq > kDwMaxQ || w.row0 + w.np > jb.NBz ||
                w.col0 + w.nq > jb.KB) { printf("\nshare out of grid\n"); return 1; }
            for (int r = 32 * w.row0; r < 32 * (w.row0 + w.np); ++r) {
                for (int cc = 32 * w.col0; cc < 32 * (w.col0 + w.nq); ++cc) dup += !written.insert({j, r, cc}).second;
                if (w.bias) dup += !written.insert({j, r, jb.KB * 32}).second;
            }
        }
        printf("\n");
    }
    long bad = 0, n = 0;
    for (int k = 0; k < p.n_red; ++k) {
        const ReduceRange& r = p.red[k];
        for (int row = 0; row < r.rows; ++row) {
            for (int col = 0; col < r.in; ++col) {
                int job = -1, sr = 0, sc = 0;
                for (int s = 0; s < r.nseg; ++s) {
                    const RedSeg& sg = r.seg[s];
                    if (col >= sg.col0 && col < sg.col0 + sg.width) { job = sg.job; sr = sg.slab_row0 + row; sc = sg.slab_col0 + col - sg.col0; }
                }
                ++n;
                if (job < 0 || !written.count({job, sr, sc})) { if (bad < 5) printf("unwritten W red %d row %d col %d job %d (%d,%d)\n", k, row, col, job, sr, sc); ++bad; }
            }
            ++n;
            if (!written.count({r.bjob, r.brow0 + row, p.job[r.bjob].KB * 32})) { if (bad < 10) printf("unwritten b red %d row %d\n", k, row); ++bad; }
        }
    }
    printf("params %ld (plan %ld) unwritten %ld doubly written %ld\n", n, (long)p.param_count, bad, dup);
    // dW workgroups per job (make_sizes): one round, every job at least one chunk, the
    // slab sets cover the largest job; uniform for 16-bit (the pipelined backward's chunks)
    long wg_bad = 0;
    for (long M : {1L, 5000L, 262144L, 786432L}) {
        const MlpSizes z = make_sizes(p, M);
        int tot = 0, mx = 0;
        printf("M %ld chunks %d max %d:", M, z.chunks, z.max_chunks);
        for (int j = 0; j < p.n_jobs; ++j) {
            printf(" %d", z.job_chunks[j]);
            tot += z.job_chunks[j];
            mx = z.job_chunks[j] > mx ? z.job_chunks[j] : mx;
            wg_bad += z.job_chunks[j] < 1 || (p.fpb == 2 && z.job_chunks[j] != z.chunks);
        }
        printf(" (sum %d)\n", tot);
        wg_bad += tot > 256 || mx != z.max_chunks;
    }
    printf("dW workgroup plan bad %ld\n", wg_bad);
    return bad != 0 || dup != 0 || n != p.param_count || wg_bad != 0;
}
