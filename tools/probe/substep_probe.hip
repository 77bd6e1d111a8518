// Probe on gfx950: latency of the BlueSky substep (substep<false> of bsg_kernels.hip) for
// one wave of real Merge aircraft (two envs, 64 lanes), one wave on the chip -- the
// single-wave regime that bounds a C4 shard (512 envs/GPU) and the kernel's critical
// path.  State comes from tools/probe/substep_probe.py (a DeviceBatch after 30 steps).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
//         -mllvm -disable-machine-licm tools/probe/substep_probe.hip -o tools/probe/substep_probe
// section marks inside substep (bsg_kernels.hip BSG_SUBSTEP_MARK): s_memtime per mark
__device__ long long g_mark[8];
#ifdef PROBE_CUT
// instruction-count builds (tools/probe/pmc_sections.sh): the substep ends at mark PROBE_CUT, so
// rocprofv3's SQ_INSTS_* of consecutive cuts give each section's dynamic instruction count
#define BSG_SUBSTEP_MARK(i) do { g_mark[i] = __builtin_amdgcn_s_memtime(); if ((i) == PROBE_CUT) return; } while (0)
#else
#define BSG_SUBSTEP_MARK(i) do { g_mark[i] = __builtin_amdgcn_s_memtime(); } while (0)
#endif
#include "../../bluesky-gym-hallucination_amd/csrc/bsg_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef PROBE_MODE
#define PROBE_MODE 0
#endif
#ifndef PROBE_HMEMO
#define PROBE_HMEMO false          // as the Merge kernel (LNAV intruders)
#endif

constexpr int NF = 12;       // lat lon alt hdg tas cas vs ax ap_trk selspd selalt selvs, + nav
constexpr int SMAX = 32;

__global__ void probe(bsg::Route route, bsg::RouteTrig rtrig, const double* st, int S, double dt, long long* cyc, double* out) {
  using namespace bsg;
  const int l = threadIdx.x;
  AC s{};
  double* f[NF] = {&s.lat, &s.lon, &s.alt, &s.hdg, &s.tas, &s.cas, &s.vs, &s.ax, &s.ap_trk,
                   &s.selspd, &s.selalt, &s.selvs};
  for (int k = 0; k < NF; ++k) *f[k] = st[k * 64 + l];
  s.nav = (int)st[NF * 64 + l];
  s.gs = s.tas; s.trk = s.hdg;
#if PROBE_MODE >= 1
  s.nav = 0;                 // LNAV off: the substep without the waypoint bearing
#endif
#if PROBE_MODE >= 2
  s.ap_trk = s.hdg;          // and no heading change: heading trig memo hits
#endif
  Memo m;
  memo_init(m, s);
  RouteRegs rt;
  rt.load(route, rtrig);
  memo_lnav(m, s, rt);
  const bool trk_ok = __ballot(!(fabs(s.ap_trk) < 360.0)) == 0;        // as propagate
  const bool fh0 = trk_ok && __ballot(!(s.hdg >= 0.0 && s.hdg <= 360.0)) == 0;
  WindDev w{};
  long long t[SMAX + 1];
  t[0] = __builtin_amdgcn_s_memtime();
  long long mk[SMAX][8];
  for (int it = 0; it < S; ++it) {
    substep<false, PROBE_HMEMO>(s, m, dt, rt, w, it == 0 ? fh0 : trk_ok);
    t[it + 1] = __builtin_amdgcn_s_memtime();
    for (int q = 0; q < 8; ++q) mk[it][q] = g_mark[q];
  }
  if (l == 0)
    for (int it = 0; it < S; ++it)
      for (int q = 0; q < 8; ++q) cyc[SMAX + it * 8 + q] = mk[it][q] - t[it];
  if (l == 0)
    for (int it = 0; it < S; ++it) cyc[it] = t[it + 1] - t[it];
  for (int k = 0; k < NF; ++k) out[k * 64 + l] = *f[k];
}

int main(int argc, char** argv) {
  if (argc < 2) { std::printf("usage: substep_probe state.bin [substeps] [dt]\n"); return 2; }
  FILE* fp = std::fopen(argv[1], "rb");
  if (!fp) return 2;
  std::vector<double> hdr(1 + 3 * BSG_MAX_ROUTE), st((NF + 1) * 64);
  if (std::fread(hdr.data(), 8, hdr.size(), fp) != hdr.size() ||
      std::fread(st.data(), 8, st.size(), fp) != st.size()) return 2;
  std::fclose(fp);
  bsg::Route route{};
  bsg::RouteTrig rtrig{};
  route.len = (int)hdr[0];
  for (int k = 0; k < BSG_MAX_ROUTE; ++k) {
    route.lat[k] = hdr[1 + k]; route.lon[k] = hdr[1 + BSG_MAX_ROUTE + k];
    route.next_qdr[k] = hdr[1 + 2 * BSG_MAX_ROUTE + k];
    // (rwgs is only a bound's centre; the per-waypoint LNAV terms as bsg_create fills them)
    bsg::sincos_t(route.lat[k] * bsg::kD2R, &rtrig.sinlat[k], &rtrig.coslat[k]);
    rtrig.lonr[k] = route.lon[k] * bsg::kD2R;
    rtrig.pnq[k] = bsg::pymod360(route.next_qdr[k]);
  }
  double *dst, *dout;
  long long* dcyc;
  if (hipMalloc(&dst, st.size() * 8) != hipSuccess || hipMalloc(&dout, NF * 64 * 8) != hipSuccess ||
      hipMalloc(&dcyc, (SMAX + SMAX * 8) * 8) != hipSuccess) return 1;
  (void)hipMemcpy(dst, st.data(), st.size() * 8, hipMemcpyHostToDevice);
  const int S = argc > 2 ? std::atoi(argv[2]) : 10;        // substeps (<= SMAX)
  const double dt = argc > 3 ? std::atof(argv[3]) : 5.0;    // simdt
  if (S < 2 || S > SMAX) return 2;
  std::vector<long long> best(S, 1LL << 62);
  for (int rep = 0; rep < 7; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, route, rtrig, dst, S, dt, dcyc, dout);
    std::vector<long long> c(S);
    (void)hipMemcpy(c.data(), dcyc, S * 8, hipMemcpyDeviceToHost);
    for (int i = 0; i < S; ++i) best[i] = c[i] < best[i] ? c[i] : best[i];
  }
  {
    std::vector<long long> c(SMAX + SMAX * 8);
    (void)hipMemcpy(c.data(), dcyc, c.size() * 8, hipMemcpyDeviceToHost);
    std::printf("section marks (cycles from substep start; 5 after qdr_x, 6 after the near-waypoint\n"
                "block, 1 after LNAV, 2 after speed/limits, 3 after the turn, 4 after the heading trig):\n");
    for (int it = 0; it < S; ++it) {
      std::printf("  substep %d:", it);
      const int order[6] = {5, 6, 1, 2, 3, 4};
      for (int q : order) std::printf(" m%d=%lld", q, c[SMAX + it * 8 + q]);
      std::printf("\n");
    }
  }
  long long tot = 0;
  std::printf("substep cycles (one wave, min of 7):");
  for (int i = 0; i < S; ++i) { std::printf(" %lld", best[i]); tot += best[i]; }
  std::printf("\nfirst %lld  mean of the rest %.0f  total %lld\n", best[0],
              (double)(tot - best[0]) / (S - 1), tot);
  return 0;
}
