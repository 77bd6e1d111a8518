// bsg_kernels.hip -- fused RL-step kernels for gfx950 (MergeEnv-v0, VerticalCREnv-v0,
// DescentEnv-v0).
//
// Mapping: one 64-lane wavefront = one workgroup = 64/GS envs; lane (g, j) owns
// aircraft j of env g (GS = next power of two >= N).  Per launch each lane
//   A. loads (or spawns) its aircraft from the [E][N] fp64 SoA arrays (coalesced),
//      applies the action (j == 0) and integrates ACTION_FREQUENCY BlueSky substeps in
//      registers (no inter-lane traffic: with RESO OFF the kinematics are per aircraft);
//   B. stages the post-step state in LDS, computes the env-layer observation, the
//      reward / termination / TimeLimit (lane j == 0), the nearest-K selection (rank by
//      LDS sweep), the intrusion mask (wave ballot) and the StateBased all-pairs CPA row
//      of aircraft j (LDS sweep over the group), reduces min separation with wave
//      shuffles, and writes every output;
//   C. (SAME_STEP autoreset) respawns finished envs and writes their reset observation;
//   and stores the state back.
// Every barrier is executed by all 64 lanes (block-uniform control flow).
#include <hip/hip_runtime.h>

#include "bsg_device.h"
#include "bsg_internal.h"

namespace bsg {

// ---- per-lane aircraft state ------------------------------------------------------------
struct AC {
  double lat, lon, alt, hdg, tas, cas, vs, ax;
  double ap_trk, selspd, selalt, selvs;
  int nav;
};

__device__ __forceinline__ void load_ac(const Buffers& b, int a, AC& s) {
  s.lat = b.lat[a]; s.lon = b.lon[a]; s.alt = b.alt[a]; s.hdg = b.hdg[a];
  s.tas = b.tas[a]; s.cas = b.cas[a]; s.vs = b.vs[a]; s.ax = b.ax[a];
  s.ap_trk = b.ap_trk[a]; s.selspd = b.selspd[a]; s.selalt = b.selalt[a]; s.selvs = b.selvs[a];
  s.nav = b.nav[a];
}

__device__ __forceinline__ void store_ac(const Buffers& b, int a, const AC& s) {
  b.lat[a] = s.lat; b.lon[a] = s.lon; b.alt[a] = s.alt; b.hdg[a] = s.hdg;
  b.tas[a] = s.tas; b.cas[a] = s.cas; b.vs[a] = s.vs; b.ax[a] = s.ax;
  b.ap_trk[a] = s.ap_trk; b.selspd[a] = s.selspd; b.selalt[a] = s.selalt; b.selvs[a] = s.selvs;
  b.nav[a] = s.nav;
}

// Traffic.cre (bluesky/traffic/traffic.py): creation state + autopilot holding it
__device__ __forceinline__ void cre(AC& s, double lat, double lon, double hdg, double alt,
                                    double spd) {
  Atmos at = vatmos(alt);
  double tas, cas;
  casormach_at(spd, at, &tas, &cas);
  s.lat = lat; s.lon = lon; s.alt = alt; s.hdg = hdg; s.tas = tas; s.cas = cas;
  s.vs = 0.0; s.ax = 0.0; s.ap_trk = hdg; s.selspd = cas; s.selalt = alt; s.selvs = 0.0;
  s.nav = 0;
}

// ---- one BlueSky substep of one aircraft (Traffic.update, wind off, RESO OFF) ---------
// oracle/bluesky_subset.py: traffic_update
__device__ __forceinline__ void substep(AC& s, double dt, const Route& rt) {
  // Autopilot.update -- LNAV direct-to + ActiveWaypoint.reached (gs = tas, trk = hdg)
  if (s.nav & 1) {
    int k = (s.nav >> 8) & 0xff;
    double qdr, dnm;
    qdrdist(s.lat, s.lon, rt.lat[k], rt.lon[k], &qdr, &dnm);
    double dist = dnm * NM;
    double nq = rt.next_qdr[k];
    double next_qdr = nq < -900.0 ? qdr : nq;
    double turnrad = s.tas * s.tas / (npmax(0.01, TAN_BANKDEF) * G0);
    double turndist = fabs(turnrad * tan((0.5 * fabs(degto180(pymod(qdr, 360.0) -
                                                                pymod(next_qdr, 360.0)))) * kD2R));
    bool close2wp = dist / npmax(0.0001, fabs(s.tas)) < 4.0;
    bool tooclose = close2wp && (fabs(degto180(pymod(s.hdg, 360.0) - pymod(qdr, 360.0))) > 90.0);
    if ((dist < turndist) || tooclose) {
      if (k >= rt.len - 1) {
        s.nav &= ~1;                       // last waypoint: LNAV off, keep commanded track
      } else {
        ++k;
        s.nav = (k << 8) | 1;
        qdrdist(s.lat, s.lon, rt.lat[k], rt.lon[k], &qdr, &dnm);
      }
    }
    if (s.nav & 1) s.ap_trk = qdr;
  }
  const double ap_vs = fabs(s.selvs) > 0.1 ? s.selvs : APVSDEF;
  const double ap_alt = s.selalt;
  const Atmos at = vatmos(s.alt);
  const double ap_tas = casormach2tas_at(s.selspd, at);
  // aporasas
  const double vs_cmd0 = fabs(ap_vs);
  const double hdg_cmd = pymod(s.ap_trk, 360.0);
  // PerfModel.limits (frozen A320 envelope)
  const double allow_h = ap_alt > HMAX ? HMAX : ap_alt;
  const Atmos ah = (allow_h == s.alt) ? at : vatmos(allow_h);
  const double intent_cas = tas2cas_at(ap_tas, ah);
  double allow_cas = intent_cas < VMIN_CAS ? VMIN_CAS : intent_cas;
  allow_cas = intent_cas > VMAX_CAS ? VMAX_CAS : allow_cas;
  double allow_tas = cas2tas_at(allow_cas, ah);
  const double snd_h = sound_at(ah);
  if (allow_tas / snd_h > MMO) allow_tas = MMO * snd_h;
  const double vs_max_with_acc = (1 - s.ax / AXMAX) * VSMAX;
  double vs_cmd = (vs_cmd0 > 0 && vs_cmd0 > VSMAX) ? vs_max_with_acc : vs_cmd0;
  vs_cmd = (vs_cmd0 < 0 && vs_cmd0 < VSMIN) ? VSMIN : vs_cmd;
  // update_airspeed
  const double delta_spd = allow_tas - s.tas;
  const bool need_ax = fabs(delta_spd) > fabs(dt * AXMAX);
  s.ax = (double)need_ax * sgn(delta_spd) * AXMAX;
  s.tas = need_ax ? s.tas + s.ax * dt : allow_tas;
  s.cas = tas2cas_at(s.tas, at);
  const double turnrate = (G0 * TAN_BANKDEF / npmax(s.tas, EPS_SPD)) * kR2D;
  const double delhdg = pymod(hdg_cmd - s.hdg + 180.0, 360.0) - 180.0;
  const bool swhdgsel = fabs(delhdg) > fabs(dt * turnrate);
  s.hdg = pymod(swhdgsel ? s.hdg + dt * turnrate * sgn(delhdg) : hdg_cmd, 360.0);
  const double delta_alt = allow_h - s.alt;
  const bool swaltsel = fabs(delta_alt) > npmax(10 * FT, fabs(2 * fabs(dt * s.vs)));
  const double target_vs = (double)swaltsel * sgn(delta_alt) * fabs(vs_cmd);
  const double delta_vs = target_vs - s.vs;
  const bool need_az = fabs(delta_vs) > 300 * FPM;
  const double az = (double)need_az * sgn(delta_vs) * (300 * FPM);
  s.vs = need_az ? s.vs + az * dt : target_vs;
  if (!isfinite(s.vs)) s.vs = 0.0;
  // update_groundspeed (no wind) + update_pos
  const double gsnorth = s.tas * cos(s.hdg * kD2R);
  const double gseast = s.tas * sin(s.hdg * kD2R);
  s.alt = swaltsel ? rint((s.alt + s.vs * dt) * 1e6) / 1e6 : allow_h;
  s.lat = s.lat + (dt * gsnorth / Rearth) * kR2D;
  const double coslat = cos(s.lat * kD2R);
  s.lon = s.lon + (dt * gseast / coslat / Rearth) * kR2D;
}

// ---- LDS staging (one wave per block; GS lanes per env) -------------------------------
struct Lds {
  double lat[64], lon[64], alt[64], hdg[64], tas[64], vs[64], u[64], v[64], d[64];
  int done[64];
};

__device__ __forceinline__ void stage(Lds& L, int lane, bool ok, const AC& s) {
  L.lat[lane] = s.lat; L.lon[lane] = s.lon; L.alt[lane] = s.alt; L.hdg[lane] = s.hdg;
  L.tas[lane] = s.tas; L.vs[lane] = s.vs;
  if (ok) {
    // StateBased: u = gs*sin(trk), v = gs*cos(trk)  (gs = tas, trk = hdg, no wind)
    double trkrad = s.hdg * kD2R;
    L.u[lane] = s.tas * sin(trkrad);
    L.v[lane] = s.tas * cos(trkrad);
  }
}

// StateBased.detect row i = lane j vs every aircraft k of the group (oracle: statebased_detect)
template <int GS>
__device__ __forceinline__ void cd_row(const Lds& L, int base, int j, int N, uint64_t* conf,
                                       uint64_t* los, double* tcpamax, double* minsep) {
  const double lati = L.lat[base + j], loni = L.lon[base + j], alti = L.alt[base + j];
  const double ui = L.u[base + j], vi = L.v[base + j], vsi = L.vs[base + j];
  const double R2 = RPZ * RPZ;
  uint64_t cm = 0, lm = 0;
  double tmax = 0.0;     // np.max(tcpa * swconfl) -- diagonal contributes 0
  double dmin = __builtin_inf();
  bool first = true;
  for (int k = 0; k < N; ++k) {
    double qdr, dnm;
    kwikqdrdist_mat(lati, loni, L.lat[base + k], L.lon[base + k], &qdr, &dnm);
    const double diag = (k == j) ? 1e9 : 0.0;
    const double dist = dnm * NM + diag;
    const double qdrrad = qdr * kD2R;
    const double dx = dist * sin(qdrrad);
    const double dy = dist * cos(qdrrad);
    const double du = L.u[base + k] - ui;
    const double dv = L.v[base + k] - vi;
    double dv2 = du * du + dv * dv;
    dv2 = fabs(dv2) < 1e-6 ? 1e-6 : dv2;
    const double vrel = sqrt(dv2);
    const double tcpa = -(du * dx + dv * dy) / dv2 + diag;
    const double dcpa2 = fabs(dist * dist - tcpa * tcpa * dv2);
    const bool swhor = dcpa2 < R2;
    const double dxinhor = sqrt(npmax(0.0, R2 - dcpa2));
    const double dtinhor = dxinhor / vrel;
    const double tinhor = swhor ? tcpa - dtinhor : 1e8;
    const double touthor = swhor ? tcpa + dtinhor : -1e8;
    const double dalt = L.alt[base + k] - alti + diag;
    double dvs = L.vs[base + k] - vsi;
    dvs = fabs(dvs) < 1e-6 ? 1e-6 : dvs;
    const double tcrosshi = (dalt + HPZ) / -dvs;
    const double tcrosslo = (dalt - HPZ) / -dvs;
    const double tinver = npmin(tcrosshi, tcrosslo);
    const double toutver = npmax(tcrosshi, tcrosslo);
    const double tin = npmax(tinver, tinhor);
    const double tout = npmin(toutver, touthor);
    const bool confl = swhor && (tin <= tout) && (tout > 0.0) && (tin < DTLOOKAHEAD) && (k != j);
    const bool lossep = (dist < RPZ) && (fabs(dalt) < HPZ);
    cm |= (uint64_t)confl << k;
    lm |= (uint64_t)lossep << k;
    const double tc = tcpa * (double)confl;
    if (first || tc > tmax) tmax = tc;
    first = false;
    if (k != j) dmin = npmin(dmin, dist);
  }
  *conf = cm; *los = lm; *tcpamax = tmax; *minsep = dmin;
}

template <int GS>
__device__ __forceinline__ uint64_t group_bits(uint64_t ballot, int g) {
  const uint64_t gm = (GS == 64) ? ~0ull : ((1ull << GS) - 1ull);
  return (ballot >> (g * GS)) & gm;
}

template <int GS>
__device__ __forceinline__ double group_min(double v) {
#pragma unroll
  for (int off = GS / 2; off > 0; off >>= 1) v = npmin(v, __shfl_xor(v, off, 64));
  return v;
}

// ---------------------------------------------------------------------------------------
// Spawn (device-side reset, K4): host parameters (parity mode) or Philox (throughput mode)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void spawn_merge(const KParams& p, int e, int j, uint32_t episode,
                                            AC& s) {
  double brg, dist;
  if (p.spawn) {
    const int W = 2 * p.N;
    brg = p.spawn[(size_t)e * W + 2 * j];
    dist = p.spawn[(size_t)e * W + 2 * j + 1];
  } else {
    U4 r = philox4x32_10((uint32_t)e, episode, (uint32_t)j, TAG_MERGE, p.seed);
    double ua = u01_53(r.x, r.y), ub = u01_53(r.z, r.w);
    const double a = -15.0, b = 15.0;                       // +-D_HEADING (merge_env.py:27)
    brg = a + (b - a) * ua;
    const double dmin = j == 0 ? 50.0 : 20.0, dmax = j == 0 ? 200.0 : 500.0;   // :21-25
    dist = dmin + (dmax - dmin) * ub;
  }
  double lat, lon;
  get_point_at_distance(p.cfg.wpt_lat[0], p.cfg.wpt_lon[0], dist, brg, &lat, &lon);
  cre(s, lat, lon, brg - 180, 10000.0, 100.0);               // merge_env.py:119,154
  if (j > 0) s.nav = 1;                                      // ADDWPT FIX; DEST RWY -> LNAV on
}

// vertical_cr_env.py:267-268 / descent_env.py:170-171 (alt_init, target_alt)
__device__ __forceinline__ void draw_alts(const KParams& p, int e, uint32_t episode, uint32_t tag,
                                          double* alt_init, double* target) {
  if (p.spawn) {
    const int W = p.spawn_width;
    *alt_init = p.spawn[(size_t)e * W + 0];
    *target = p.spawn[(size_t)e * W + 1];
  } else {
    U4 r = philox4x32_10((uint32_t)e, episode, 0u, tag, p.seed);
    int64_t ai = randint_u32(r.x, 2000, 4000);
    int64_t dt = randint_u32(r.y, -500, 500);
    *alt_init = (double)ai;
    *target = (double)(ai + dt);
  }
}

__device__ __forceinline__ void spawn_vertical(const KParams& p, int e, int j, uint32_t episode,
                                               AC& s, double* target_out) {
  double alt_init, target;
  draw_alts(p, e, episode, TAG_VERT, &alt_init, &target);
  *target_out = target;
  // ownship: cre('KL001', acalt=alt_init, acspd=150) at default 52N 4E, hdg 0
  cre(s, 52.0, 4.0, 0.0, alt_init, 150.0);
  if (j == 0) return;
  const double gsref = s.tas;       // ownship gs after cre (computed identically per lane)
  double dpsi, cpa, tlosh, dH;
  if (p.spawn) {
    const double* q = p.spawn + (size_t)e * p.spawn_width + 2 + 4 * (j - 1);
    dpsi = q[0]; cpa = q[1]; tlosh = q[2]; dH = q[3];
  } else {
    // distributions of vertical_cr_env.py:187-195, Philox multiply-shift randint
    U4 r = philox4x32_10((uint32_t)e, episode, (uint32_t)j, TAG_VERT, p.seed);
    const double altitude = alt_init;
    dpsi = (double)randint_u32(r.x, 45, 315);
    cpa = (double)randint_u32(r.y, 0, 5);
    const int64_t hi_t = (int64_t)(((200 * 0.9) * 1000) / gsref);
    const int64_t tl = randint_u32(r.z, 100, hi_t);
    tlosh = (double)tl;
    const double average_tod = (200.0 * 1000 / gsref) - 2 * target / 12.5;
    int64_t lo, hi;
    if ((double)tl > average_tod) {
      lo = (int64_t)(-altitude + 500); hi = (int64_t)((target - altitude) + 100);
    } else {
      lo = (int64_t)((target - altitude) - 500); hi = (int64_t)((target - altitude) + 500);
    }
    dH = (double)randint_u32(r.w, lo, hi);
  }
  // Traffic.creconfs (spd=None branch), oracle/bluesky_subset.py: creconfs_params
  const double trkref = 0.0 * kD2R;
  const double cpam = cpa * NM;
  const double pzr = RPZ, pzh = HPZ;
  const double trk = trkref + dpsi * kD2R;
  const double acalt = alt_init + dH;
  const double tlosv = 100000000000.0;
  const double acvs = 0.0 - sgn(dH) * (fabs(dH) - pzh) / tlosv;
  const double gsn = gsref * cos(trk), gse = gsref * sin(trk);
  const double vreln = gsref * cos(trkref) - gsn, vrele = gsref * sin(trkref) - gse;
  const double vrel = sqrt(vreln * vreln + vrele * vrele);
  const double drelcpa = tlosh * vrel + (cpam > pzr ? 0.0 : sqrt(pzr * pzr - cpam * cpam));
  const double dist = sqrt(drelcpa * drelcpa + cpam * cpam);
  const double rd = drelcpa / dist;
  const double rx = cpam / dist;
  const double brn = atan2(-rx * vreln + rd * vrele, rd * vreln + rx * vrele) * kR2D;
  double aclat, aclon;
  kwikpos(52.0, 4.0, brn, dist / NM, &aclat, &aclon);
  const double acspd = tas2cas_at(sqrt(gsn * gsn + gse * gse), vatmos(acalt));
  const double achdg = atan2(gse, gsn) * kR2D;
  cre(s, aclat, aclon, achdg, acalt, acspd);
  s.vs = acvs;
  s.alt = alt_init + dH;            // vertical_cr_env.py:199
  s.selalt = alt_init + dH;         // :200 selaltcmd(i+1, alt + dH, 0)
  s.selvs = acvs;
}

// ---------------------------------------------------------------------------------------
// Observation / reward per env kind.  Values are computed into registers first; the
// done flag is published through LDS; then outputs are written.
// ---------------------------------------------------------------------------------------
struct EnvScalars {
  int step_count, flags, wpt_reach, faf_reached, total_intr;
  uint32_t episode;
  double total_reward, drift_sum, target_alt, final_alt;
};

__device__ __forceinline__ void load_env(const Buffers& b, int e, EnvScalars& v) {
  v.step_count = b.step_count[e]; v.flags = b.flags[e]; v.wpt_reach = b.wpt_reach[e];
  v.faf_reached = b.faf_reached[e]; v.total_intr = b.total_intrusions[e];
  v.episode = b.episode[e]; v.total_reward = b.total_reward[e]; v.drift_sum = b.drift_sum[e];
  v.target_alt = b.target_alt[e]; v.final_alt = b.final_altitude[e];
}

__device__ __forceinline__ void store_env(const Buffers& b, int e, const EnvScalars& v) {
  b.step_count[e] = v.step_count; b.flags[e] = v.flags; b.wpt_reach[e] = v.wpt_reach;
  b.faf_reached[e] = v.faf_reached; b.total_intrusions[e] = v.total_intr;
  b.episode[e] = v.episode; b.total_reward[e] = v.total_reward; b.drift_sum[e] = v.drift_sum;
  b.target_alt[e] = v.target_alt; b.final_altitude[e] = v.final_alt;
}

__device__ __forceinline__ void reset_scalars(EnvScalars& v, double target) {
  v.step_count = 0; v.flags = 0; v.wpt_reach = 0; v.faf_reached = 0; v.total_intr = 0;
  v.total_reward = 0.0; v.drift_sum = 0.0; v.target_alt = target; v.final_alt = 0.0;
  v.episode += 1;
}

template <int KIND, int GS>
__global__ __launch_bounds__(64) void step_kernel(KParams p) {
  __shared__ Lds L;
  const int lane = threadIdx.x;
  const int g = lane / GS;
  const int j = lane % GS;
  const int base = g * GS;
  const int e = blockIdx.x * (64 / GS) + g;
  const int N = p.N;
  const bool env_ok = e < p.E;
  const bool ok = env_ok && j < N;
  const size_t a = (size_t)e * N + j;
  const Buffers& b = p.b;
  const int O = p.obs_dim;

  EnvScalars ev = {};
  if (env_ok) load_env(b, e, ev);
  bool resetting = false;
  if (env_ok) {
    if (p.mode == MODE_RESET) resetting = p.env_mask ? (p.env_mask[e] != 0) : true;
    else resetting = (p.cfg.autoreset_mode == BSG_AUTORESET_NEXT_STEP) && (ev.flags & 1);
  }
  const bool stepping = env_ok && p.mode == MODE_STEP && !resetting;
  const bool active = resetting || stepping;   // env produces outputs this launch

  // ---------------- A: spawn or propagate -----------------------------------------
  AC s = {};
  double new_target = ev.target_alt;
  if (ok) {
    if (resetting) {
      if constexpr (KIND == BSG_ENV_MERGE) spawn_merge(p, e, j, ev.episode, s);
      else if constexpr (KIND == BSG_ENV_VERTICAL_CR) spawn_vertical(p, e, j, ev.episode, s, &new_target);
      else {
        double alt_init;
        draw_alts(p, e, ev.episode, TAG_DESC, &alt_init, &new_target);
        cre(s, 52.0, 4.0, 0.0, alt_init, 150.0);
      }
    } else {
      load_ac(b, (int)a, s);
    }
    if (stepping) {
      if (j == 0) {
        if constexpr (KIND == BSG_ENV_MERGE) {
          // merge_env.py:286-293 -> HDG / SPD stack commands
          const double dh = p.actions[(size_t)e * 2 + 0] * 15;
          const double dv = p.actions[(size_t)e * 2 + 1] * 20;
          const double heading_new = bound180(s.hdg + dh);
          const double speed_new = (s.cas + dv) * 1.94384;
          s.ap_trk = heading_new;
          s.nav &= ~1;
          s.selspd = speed_new >= 1.0 ? speed_new * KTS : speed_new;
        } else {
          // vertical_cr_env.py:242-256 / descent_env.py:146-160
          const double act = p.actions[e] * 12.5;
          if (act >= 0) { s.selalt = 1000000; s.selvs = act; }
          else if (act < 0) { s.selalt = 0; s.selvs = act; }
        }
      }
      for (int it = 0; it < p.cfg.action_frequency; ++it) substep(s, p.cfg.simdt, p.route);
    }
  }
  if (resetting && j == 0) reset_scalars(ev, new_target);

  // ---------------- B: observation, reward, CD -----------------------------------------
  stage(L, lane, ok, s);
  __syncthreads();

  bool done = false;
  float reward = 0.0f;
  bool term = false, trunc = false;
  // per-lane obs values
  double o0 = 0, o1 = 0, o2 = 0, o3 = 0, o4 = 0, o5 = 0, o6 = 0;
  int rank = 0x7fffffff;
  bool intr = false;
  if constexpr (KIND == BSG_ENV_MERGE) {
    const double lat0 = L.lat[base], lon0 = L.lon[base], hdg0 = L.hdg[base], tas0 = L.tas[base];
    if (ok && j > 0) {
      // merge_env.py:195-218
      const double dmat = kwikdist_mat(lat0, lon0, s.lat, s.lon);
      double brg, dist;
      kwikqdrdist(lat0, lon0, s.lat, s.lon, &brg, &dist);
      const double vx = cos(hdg0 * kD2R) * tas0;
      const double vy = sin(hdg0 * kD2R) * tas0;
      const double x_r = (dist * 1.852 * 1000) * cos(brg * kD2R);
      const double y_r = (dist * 1.852 * 1000) * sin(brg * kD2R);
      const double vx_int = cos(s.hdg * kD2R) * s.tas;
      const double vy_int = sin(s.hdg * kD2R) * s.tas;
      const double vx_r = vx_int - vx, vy_r = vy_int - vy;
      const double track = atan2(vy_r, vx_r);
      o0 = x_r; o1 = y_r; o2 = vx_r; o3 = vy_r; o4 = cos(track); o5 = sin(track); o6 = dmat;
      intr = dist < 4;                                        // _check_intrusion :280-281
      L.d[lane] = dmat;
    } else {
      L.d[lane] = __builtin_inf();
    }
  } else if constexpr (KIND == BSG_ENV_VERTICAL_CR) {
    if (ok && j > 0) {
      // vertical_cr_env.py:133-156
      const double lat0 = L.lat[base], lon0 = L.lon[base], hdg0 = L.hdg[base];
      const double alt0 = L.alt[base], vs0 = L.vs[base], gs0 = L.tas[base];
      double qdr, dis;
      kwikqdrdist(lat0, lon0, s.lat, s.lon, &qdr, &dis);
      const double bearing = bound180(hdg0 - qdr);
      const double hd = hdg0 - s.hdg;
      o0 = dis * 1.852;                                       // intruder_distance (km)
      o1 = cos(bearing * kD2R);
      o2 = sin(bearing * kD2R);
      o3 = s.alt - alt0;                                      // altitude_difference
      o4 = -cos(hd * kD2R) * s.tas;                           // x_difference_speed
      o5 = gs0 - sin(hd * kD2R) * s.tas;                      // y_difference_speed
      o6 = s.vs - vs0;                                        // z_difference_speed
      intr = (dis < 5) && (fabs(alt0 - s.alt) < 1000 * 0.3048);   // :235-237
    }
  }
  __syncthreads();
  if constexpr (KIND == BSG_ENV_MERGE) {
    if (ok && j > 0) {
      const double dj = L.d[lane];
      int r = 0;
      for (int k = 1; k < N; ++k) {
        const double dk = L.d[base + k];
        r += (dk < dj) || (dk == dj && k < j);
      }
      rank = r;
    }
  }
  const uint64_t ib = group_bits<GS>(__ballot(ok && stepping && intr), g);
  const int nintr = __popcll(ib);

  // CD: StateBased all-pairs CPA row of aircraft j
  uint64_t cmask = 0, lmask = 0;
  double tmax = 0.0, msep = __builtin_inf();
  if (p.cfg.compute_cd && KIND != BSG_ENV_DESCENT) {
    if (ok) cd_row<GS>(L, base, j, N, &cmask, &lmask, &tmax, &msep);
    msep = group_min<GS>(ok ? msep : __builtin_inf());
  }

  // lane 0: scalar obs, reward, termination (per env)
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0;
  if (ok && j == 0) {
    if constexpr (KIND == BSG_ENV_MERGE) {
      // merge_env.py:175-191 (obs uses wpt_reach BEFORE the reward update)
      const int wr = ev.wpt_reach;
      double wqdr, wdist;
      kwikqdrdist(s.lat, s.lon, p.cfg.wpt_lat[wr == 0 ? 0 : 1], p.cfg.wpt_lon[wr == 0 ? 0 : 1],
                  &wqdr, &wdist);
      const double drift = bound180(s.hdg - wqdr);
      s0 = s.tas; s1 = cos(drift * kD2R); s2 = (double)wr; s3 = sin(drift * kD2R); s4 = wdist / 250;
      if (stepping) {
        // _check_waypoint :257-268
        int reach = 0, d = 0;
        if (wdist < 10 && wr != 1) { ev.wpt_reach = 1; ev.faf_reached = 1; reach = 1; }
        else if (wdist < 2 * 10 && wr == 1) { ev.faf_reached = 2; d = 1; }
        // _check_drift :270-273 ; _check_intrusion :275-284
        const double dd = fabs(drift * kD2R);
        const double r = ((double)reach + dd * -0.1) + (double)(nintr * -1);
        ev.drift_sum += dd;
        ev.total_intr += nintr;
        ev.total_reward += r;
        reward = (float)r;
        term = d != 0;
      }
    } else {
      // vertical_cr_env.py:129-181 / descent_env.py:100-117
      const double altitude = s.alt, vz = s.vs;
      const double runway_distance = 200 - kwikdist(52.0, 4.0, s.lat, s.lon) * 1.852;
      s0 = (altitude - 1500) / 3000; s1 = (vz - 0) / 5; s2 = (ev.target_alt - 1500) / 3000;
      s3 = (runway_distance - 100) / 200;
      if (stepping) {
        // _get_reward (vertical_cr_env.py:213-228 / descent_env.py:128-144)
        double alt_pen;
        int d = 0;
        if (runway_distance > 0 && altitude > 0) {
          alt_pen = fabs(ev.target_alt - altitude) * (-5.0 / 3000);
        } else if (altitude <= 0) {
          alt_pen = -100; ev.final_alt = -100; d = 1;
        } else {
          alt_pen = altitude * (-50.0 / 3000); ev.final_alt = altitude; d = 1;
        }
        const double r = alt_pen + (double)(nintr * -50);
        ev.total_intr += nintr;
        ev.total_reward += r;
        reward = (float)r;
        term = d != 0;
      }
    }
    if (stepping) {
      ev.step_count += 1;
      trunc = p.cfg.max_episode_steps > 0 && ev.step_count >= p.cfg.max_episode_steps;
      done = term || trunc;
    }
    L.done[base] = done ? 1 : 0;
  }
  __syncthreads();
  done = env_ok && (L.done[base] != 0);
  const bool same_step_reset = done && p.cfg.autoreset_mode == BSG_AUTORESET_SAME_STEP;

  // ---- write outputs ----
  if (active && ok) {
    float* obs = b.obs + (size_t)e * O;
    float* fobs = same_step_reset ? b.final_obs + (size_t)e * O : nullptr;
    float* lrn = (b.learner && !same_step_reset) ? b.learner + (size_t)e * (O + 3) : nullptr;
    auto put = [&](int off, double v) {
      obs[off] = (float)v;
      if (fobs) fobs[off] = (float)v;
      if (lrn) lrn[off] = (float)v;
    };
    if constexpr (KIND == BSG_ENV_MERGE) {
      const int K = p.K;
      if (j == 0) {
        put(0, s0);                         // airspeed
        put(1, s1);                         // cos(drift)
        put(2 + 2 * K, s2);                 // faf_reached
        put(3 + 2 * K, s3);                 // sin(drift)
        put(4 + 5 * K, s4);                 // waypoint_dist
      } else if (rank < K) {
        put(2 + rank, o4);                  // cos(track)
        put(2 + K + rank, o6 / 250);        // distances
        put(4 + 2 * K + rank, o5);          // sin(track)
        put(4 + 3 * K + rank, o2 / 150);    // vx_r
        put(4 + 4 * K + rank, o3 / 150);    // vy_r
        put(5 + 5 * K + rank, o0 / 1000000);// x_r
        put(5 + 6 * K + rank, o1 / 1000000);// y_r
        b.topk[(size_t)e * K + rank] = j;
      }
    } else if constexpr (KIND == BSG_ENV_VERTICAL_CR) {
      const int NI = N - 1;
      if (j == 0) {
        put(0, s0);                         // altitude
        put(1 + 3 * NI, s3);                // runway_distance
        put(2 + 4 * NI, s2);                // target_altitude
        put(3 + 4 * NI, s1);                // vz
      } else {
        const int i = j - 1;
        put(1 + i, o3 / 3000);              // altitude_difference
        put(1 + NI + i, o1);                // cos_difference_pos
        put(1 + 2 * NI + i, o0 / 200);      // intruder_distance
        put(2 + 3 * NI + i, o2);            // sin_difference_pos
        put(4 + 4 * NI + i, o4 / 150);      // x_difference_speed
        put(4 + 5 * NI + i, o5 / 150);      // y_difference_speed
        put(4 + 6 * NI + i, o6);            // z_difference_speed
      }
    } else {
      if (j == 0) { put(0, s0); put(1, s3); put(2, s2); put(3, s1); }
    }
    if (j == 0) {
      b.reward[e] = reward;
      b.terminated[e] = term ? 1 : 0;
      b.truncated[e] = trunc ? 1 : 0;
      if (b.learner) {
        float* row = b.learner + (size_t)e * (O + 3);
        row[O] = reward;
        row[O + 1] = term ? 1.0f : 0.0f;
        row[O + 2] = trunc ? 1.0f : 0.0f;
      }
      if (b.intr_mask) b.intr_mask[e] = ib;
      if (done && b.ep_info) {
        double* info = b.ep_info + (size_t)e * 4;
        info[0] = ev.total_reward;
        info[1] = (double)ev.total_intr;
        if constexpr (KIND == BSG_ENV_MERGE) {
          info[2] = (double)ev.faf_reached;
          info[3] = ev.drift_sum / (double)ev.step_count;
        } else {
          info[2] = ev.final_alt;
          info[3] = 0.0;
        }
      }
    }
    if (p.cfg.compute_cd && KIND != BSG_ENV_DESCENT) {
      b.conf_mask[a] = cmask;
      b.los_mask[a] = lmask;
      b.tcpamax[a] = (float)tmax;
      if (j == 0) b.min_sep[e] = (float)msep;
    }
  }
  if (stepping && j == 0 && p.cfg.autoreset_mode == BSG_AUTORESET_NEXT_STEP && done) ev.flags |= 1;

  // ---------------- C: SAME_STEP autoreset ---------------------------------------------
  if (p.cfg.autoreset_mode == BSG_AUTORESET_SAME_STEP && __syncthreads_or(same_step_reset)) {
    double tgt = ev.target_alt;
    if (same_step_reset && ok) {
      if constexpr (KIND == BSG_ENV_MERGE) spawn_merge(p, e, j, ev.episode, s);
      else if constexpr (KIND == BSG_ENV_VERTICAL_CR) spawn_vertical(p, e, j, ev.episode, s, &tgt);
      else {
        double alt_init;
        draw_alts(p, e, ev.episode, TAG_DESC, &alt_init, &tgt);
        cre(s, 52.0, 4.0, 0.0, alt_init, 150.0);
      }
    }
    if (same_step_reset && j == 0) reset_scalars(ev, tgt);
    stage(L, lane, ok, s);
    __syncthreads();
    if constexpr (KIND == BSG_ENV_MERGE) {
      const double lat0 = L.lat[base], lon0 = L.lon[base], hdg0 = L.hdg[base], tas0 = L.tas[base];
      if (same_step_reset && ok && j > 0) {
        const double dmat = kwikdist_mat(lat0, lon0, s.lat, s.lon);
        double brg, dist;
        kwikqdrdist(lat0, lon0, s.lat, s.lon, &brg, &dist);
        const double vx = cos(hdg0 * kD2R) * tas0, vy = sin(hdg0 * kD2R) * tas0;
        const double vx_r = cos(s.hdg * kD2R) * s.tas - vx, vy_r = sin(s.hdg * kD2R) * s.tas - vy;
        const double track = atan2(vy_r, vx_r);
        o0 = (dist * 1.852 * 1000) * cos(brg * kD2R); o1 = (dist * 1.852 * 1000) * sin(brg * kD2R);
        o2 = vx_r; o3 = vy_r; o4 = cos(track); o5 = sin(track); o6 = dmat;
        L.d[lane] = dmat;
      } else {
        L.d[lane] = __builtin_inf();
      }
    } else if constexpr (KIND == BSG_ENV_VERTICAL_CR) {
      if (same_step_reset && ok && j > 0) {
        const double lat0 = L.lat[base], lon0 = L.lon[base], hdg0 = L.hdg[base];
        const double alt0 = L.alt[base], vs0 = L.vs[base], gs0 = L.tas[base];
        double qdr, dis;
        kwikqdrdist(lat0, lon0, s.lat, s.lon, &qdr, &dis);
        const double bearing = bound180(hdg0 - qdr);
        const double hd = hdg0 - s.hdg;
        o0 = dis * 1.852; o1 = cos(bearing * kD2R); o2 = sin(bearing * kD2R); o3 = s.alt - alt0;
        o4 = -cos(hd * kD2R) * s.tas; o5 = gs0 - sin(hd * kD2R) * s.tas; o6 = s.vs - vs0;
      }
    }
    __syncthreads();
    if (same_step_reset && ok) {
      float* obs = b.obs + (size_t)e * O;
      float* lrn = b.learner ? b.learner + (size_t)e * (O + 3) : nullptr;
      auto put = [&](int off, double v) {
        obs[off] = (float)v;
        if (lrn) lrn[off] = (float)v;
      };
      if constexpr (KIND == BSG_ENV_MERGE) {
        const int K = p.K;
        if (j == 0) {
          double wqdr, wdist;
          kwikqdrdist(s.lat, s.lon, p.cfg.wpt_lat[0], p.cfg.wpt_lon[0], &wqdr, &wdist);
          const double drift = bound180(s.hdg - wqdr);
          put(0, s.tas); put(1, cos(drift * kD2R)); put(2 + 2 * K, 0.0);
          put(3 + 2 * K, sin(drift * kD2R)); put(4 + 5 * K, wdist / 250);
        } else {
          const double dj = L.d[lane];
          int r = 0;
          for (int k = 1; k < N; ++k) {
            const double dk = L.d[base + k];
            r += (dk < dj) || (dk == dj && k < j);
          }
          if (r < K) {
            put(2 + r, o4); put(2 + K + r, o6 / 250); put(4 + 2 * K + r, o5);
            put(4 + 3 * K + r, o2 / 150); put(4 + 4 * K + r, o3 / 150);
            put(5 + 5 * K + r, o0 / 1000000); put(5 + 6 * K + r, o1 / 1000000);
          }
        }
      } else if constexpr (KIND == BSG_ENV_VERTICAL_CR) {
        const int NI = N - 1;
        if (j == 0) {
          const double rd = 200 - kwikdist(52.0, 4.0, s.lat, s.lon) * 1.852;
          put(0, (s.alt - 1500) / 3000); put(1 + 3 * NI, (rd - 100) / 200);
          put(2 + 4 * NI, (ev.target_alt - 1500) / 3000); put(3 + 4 * NI, (s.vs - 0) / 5);
        } else {
          const int i = j - 1;
          put(1 + i, o3 / 3000); put(1 + NI + i, o1); put(1 + 2 * NI + i, o0 / 200);
          put(2 + 3 * NI + i, o2); put(4 + 4 * NI + i, o4 / 150);
          put(4 + 5 * NI + i, o5 / 150); put(4 + 6 * NI + i, o6);
        }
      } else {
        if (j == 0) {
          const double rd = 200 - kwikdist(52.0, 4.0, s.lat, s.lon) * 1.852;
          put(0, (s.alt - 1500) / 3000); put(1, (rd - 100) / 200);
          put(2, (ev.target_alt - 1500) / 3000); put(3, (s.vs - 0) / 5);
        }
      }
    }
  }

  // ---------------- store ----------------------------------------------------------------
  if (active && ok) store_ac(b, (int)a, s);
  if (active && j == 0) store_env(b, e, ev);
}

// ---------------------------------------------------------------------------------------
template <int KIND>
static hipError_t launch_kind(const KParams& p, hipStream_t st) {
  int gs = 1;
  while (gs < p.N) gs <<= 1;
  const int epb = 64 / gs;
  const int grid = (p.E + epb - 1) / epb;
  switch (gs) {
#define BSG_CASE(G) \
    case G: hipLaunchKernelGGL((step_kernel<KIND, G>), dim3(grid), dim3(64), 0, st, p); break;
    BSG_CASE(1) BSG_CASE(2) BSG_CASE(4) BSG_CASE(8) BSG_CASE(16) BSG_CASE(32) BSG_CASE(64)
#undef BSG_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_step(const KParams& p, hipStream_t st) {
  switch (p.cfg.env_kind) {
    case BSG_ENV_MERGE: return launch_kind<BSG_ENV_MERGE>(p, st);
    case BSG_ENV_VERTICAL_CR: return launch_kind<BSG_ENV_VERTICAL_CR>(p, st);
    case BSG_ENV_DESCENT: return launch_kind<BSG_ENV_DESCENT>(p, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace bsg
