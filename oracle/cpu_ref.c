/* CPU restatement of the Chorowski-baseline training step in plain C (fp32, OpenMP over utterances).
 *
 * TEST / MEASUREMENT INFRASTRUCTURE, not the product: bench.py's cpu_baseline leg times it (kind "port": it is a
 * C port of the reference algorithm, not Torch7), and tests/test_cpu_ref.py checks it against the float64 NumPy
 * oracle (oracle/s2s_oracle.py).  Nothing under seq2seq-attention-asr_amd/ links or loads it.
 *
 * Reference semantics (timit/timit.lua:240-295): every utterance is forwarded and back-propagated ALONE (B = 1,
 * 2-D tensors, per-time-step matrix-vector products as the reference's nn modules run them), gradients summed
 * over the minibatch, then scaled by 1/B.  Each function follows the oracle function named in its comment, which
 * cites the Lua lines:
 *   gru_fwd / gru_bwd          oracle gru_seq_fwd / gru_seq_bwd      (GRU.lua:16-38, RNN.lua:120-201)
 *   encoder                     oracle encoder_fwd / encoder_bwd      (timit/model_chorowski_baseline.lua:20-34)
 *   attention_fwd / _bwd        oracle attention_fwd / attention_bwd  (Attention.lua:51-184, RNNAttention.lua:144-253,
 *                               MonotonicAlignment.lua:19-77, Maxout.lua:14-18)
 *   s2s_cpu_step                oracle training_step                  (timit/timit.lua:262-295)
 * Content attention with the GRU decoder (the Chorowski models); optional nn.Dropout masks on the decoder MLP
 * input (model_chorowski_baseline_dropout.lua).  Parameters: the flat layout of DESIGN.md §3 (param_shapes).
 *
 * Build: make -C oracle  (-O3 -march=x86-64-v4 -fopenmp; the GPU box's EPYC 9575F and this container's Xeon both
 * have AVX-512 F/BW/CD/DQ/VL).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  int F, Hh, Ho, nl, Sc, S, O, M, k;  /* input, hidden / top-layer units, layers, score, state, output, mlp, window */
  float penalty;
} s2s_cpu_cfg;

/* ------------------------------------------------------------------ small dense helpers (row-major) */
/* y (n) = W (n x m, ld) x (m) [+ y if acc] */
static void mv(const float* restrict W, long ld, int n, int m, const float* restrict x, float* restrict y, int acc) {
  for (int i = 0; i < n; ++i) {
    const float* w = W + (long)i * ld;
    float s = 0.f;
    for (int j = 0; j < m; ++j) s += w[j] * x[j];
    y[i] = acc ? y[i] + s : s;
  }
}
/* y (m) += W^T (m x n) x (n) */
static void mtv(const float* restrict W, long ld, int n, int m, const float* restrict x, float* restrict y) {
  for (int i = 0; i < n; ++i) {
    const float xi = x[i];
    if (xi == 0.f) continue;
    const float* w = W + (long)i * ld;
    for (int j = 0; j < m; ++j) y[j] += xi * w[j];
  }
}
/* G (n x m, ld) += s * a (n) b^T (m) */
static void ger(float* restrict G, long ld, int n, int m, float s, const float* restrict a, const float* restrict b) {
  for (int i = 0; i < n; ++i) {
    const float ai = s * a[i];
    if (ai == 0.f) continue;
    float* g = G + (long)i * ld;
    for (int j = 0; j < m; ++j) g[j] += ai * b[j];
  }
}
static float sigm(float v) { return 1.f / (1.f + expf(-v)); }

/* ------------------------------------------------------------------ flat parameter layout */
typedef struct {
  long enc[8][2][3]; /* layer, dir, gate (Wz Wr Wh) */
  long V, Ws, bs, we, Wy, by, Wc, bc, Wd, bd, dWz, dWr, dWh, Wm, bm, Wo, bo, total;
} layout;
static layout layout_of(const s2s_cpu_cfg* c) {
  layout P;
  long off = 0;
  int D = c->F;
  for (int l = 0; l < c->nl; ++l) {
    const int H = l == c->nl - 1 ? c->Ho : c->Hh;
    for (int d = 0; d < 2; ++d)
      for (int g = 0; g < 3; ++g) {
        P.enc[l][d][g] = off;
        off += (long)H * (H + D);
      }
    D = 2 * H;
  }
  const int A = 2 * c->Ho, S = c->S, Sc = c->Sc, O = c->O, Mk = c->M * c->k;
  P.V = off; off += (long)Sc * A;
  P.Ws = off; off += (long)Sc * S;
  P.bs = off; off += Sc;
  P.we = off; off += Sc;
  P.Wy = off; off += (long)S * O;
  P.by = off; off += S;
  P.Wc = off; off += (long)S * A;
  P.bc = off; off += S;
  P.Wd = off; off += (long)S * 2 * S;
  P.bd = off; off += S;
  P.dWz = off; off += (long)S * 2 * S;
  P.dWr = off; off += (long)S * 2 * S;
  P.dWh = off; off += (long)S * 2 * S;
  P.Wm = off; off += (long)Mk * (S + A);
  P.bm = off; off += Mk;
  P.Wo = off; off += (long)O * c->M;
  P.bo = off; off += O;
  P.total = off;
  return P;
}
long s2s_cpu_param_count(const s2s_cpu_cfg* c) { return layout_of(c).total; }

/* ------------------------------------------------------------------ GRU over a sequence (oracle gru_seq_fwd / _bwd) */
/* x (L x D), y (L x ldy) columns [0, H); saved sv (L x 4H): z | r | hh | hprev */
static void gru_fwd(const float* x, int L, int D, int H, const float* Wz, const float* Wr, const float* Wh, int rev,
                    float* y, int ldy, float* sv, float* tmp) {
  float* h = tmp;              /* H */
  float* hx = tmp + H;         /* H + D */
  float* a = hx + H + D;       /* H */
  memset(h, 0, sizeof(float) * H);
  for (int q = 0; q < L; ++q) {
    const int t = rev ? L - 1 - q : q;
    const float* xt = x + (long)t * D;
    float* s = sv + (long)t * 4 * H;
    memcpy(hx, h, sizeof(float) * H);
    memcpy(hx + H, xt, sizeof(float) * D);
    mv(Wz, H + D, H, H + D, hx, a, 0);
    for (int i = 0; i < H; ++i) s[i] = sigm(a[i]);
    mv(Wr, H + D, H, H + D, hx, a, 0);
    for (int i = 0; i < H; ++i) s[H + i] = sigm(a[i]);
    for (int i = 0; i < H; ++i) hx[i] = s[H + i] * h[i];
    mv(Wh, H + D, H, H + D, hx, a, 0);
    for (int i = 0; i < H; ++i) {
      s[2 * H + i] = tanhf(a[i]);
      s[3 * H + i] = h[i];
      h[i] = (1.f - s[i]) * h[i] + s[i] * s[2 * H + i];
      y[(long)t * ldy + i] = h[i];
    }
  }
}
/* dy (L x lddy) columns [0, H); dx (L x D) += ; gradients G* += scale * ... */
static void gru_bwd(const float* x, int L, int D, int H, const float* Wz, const float* Wr, const float* Wh, int rev,
                    const float* sv, const float* dy, int lddy, float* dx, float* GWz, float* GWr, float* GWh,
                    float scale, float* tmp) {
  float* dnext = tmp;          /* H */
  float* dhp = dnext + H;      /* H */
  float* dah = dhp + H;        /* H */
  float* daz = dah + H;        /* H */
  float* dar = daz + H;        /* H */
  float* v = dar + H;          /* H + D */
  float* drhx = v + H + D;     /* H + D */
  memset(dnext, 0, sizeof(float) * H);
  for (int q = 0; q < L; ++q) {
    const int t = rev ? q : L - 1 - q;
    const float* xt = x + (long)t * D;
    const float* s = sv + (long)t * 4 * H;
    const float *z = s, *r = s + H, *hh = s + 2 * H, *hp = s + 3 * H;
    for (int i = 0; i < H; ++i) {
      const float dh = dy[(long)t * lddy + i] + dnext[i];
      const float dz = dh * (hh[i] - hp[i]);
      dah[i] = dh * z[i] * (1.f - hh[i] * hh[i]);
      dhp[i] = dh * (1.f - z[i]);
      daz[i] = dz * z[i] * (1.f - z[i]);
    }
    for (int i = 0; i < H; ++i) v[i] = r[i] * hp[i];
    memcpy(v + H, xt, sizeof(float) * D);
    ger(GWh, H + D, H, H + D, scale, dah, v);
    memset(drhx, 0, sizeof(float) * (H + D));
    mtv(Wh, H + D, H, H + D, dah, drhx);
    for (int i = 0; i < H; ++i) {
      const float dr = drhx[i] * hp[i];
      dhp[i] += drhx[i] * r[i];
      dar[i] = dr * r[i] * (1.f - r[i]);
    }
    memcpy(v, hp, sizeof(float) * H);
    ger(GWz, H + D, H, H + D, scale, daz, v);
    ger(GWr, H + D, H, H + D, scale, dar, v);
    /* drhx[H:] holds dx from the candidate; add Wz^T daz + Wr^T dar */
    memset(v, 0, sizeof(float) * (H + D));
    mtv(Wz, H + D, H, H + D, daz, v);
    mtv(Wr, H + D, H, H + D, dar, v);
    for (int i = 0; i < H; ++i) dnext[i] = dhp[i] + v[i];
    float* dxt = dx + (long)t * D;
    for (int j = 0; j < D; ++j) dxt[j] += drhx[H + j] + v[H + j];
  }
}

/* ------------------------------------------------------------------ one utterance */
typedef struct {
  float *ws, *alpha, *c, *cin, *yin, *d, *sp, *ind, *m, *logp, *v, *z, *r, *hh;
  int* am;
} dec_cache;

/* oracle training_step for B = 1: grads (flat) += scale * d nll / d params; returns nll (/T when normalize) */
static float utterance(const s2s_cpu_cfg* c, const layout* P, const float* W, const float* x, const int* lab, int L,
                       int T, const float* mask, int normalize, float* G, float scale) {
  const int A = 2 * c->Ho, S = c->S, Sc = c->Sc, O = c->O, M = c->M, k = c->k, Mk = M * k, nl = c->nl;
  int Hmax = c->Hh > c->Ho ? c->Hh : c->Ho, Dmax = c->F > 2 * Hmax ? c->F : 2 * Hmax;
  int big = Sc > A ? Sc : A;
  if (big < S + A) big = S + A;
  if (big < Mk) big = Mk;
  if (big < 2 * S) big = 2 * S;
  /* ---- encoder forward (oracle encoder_fwd) */
  float** inp = (float**)malloc(sizeof(float*) * (nl + 1));
  float** svs = (float**)malloc(sizeof(float*) * nl * 2);
  float* tmp = (float*)malloc(sizeof(float) * (8 * (Hmax + Dmax) + 8 * big + 64));
  inp[0] = (float*)x;
  int D = c->F;
  for (int l = 0; l < nl; ++l) {
    const int H = l == nl - 1 ? c->Ho : c->Hh;
    inp[l + 1] = (float*)malloc(sizeof(float) * (long)L * 2 * H);
    for (int dir = 0; dir < 2; ++dir) {
      svs[2 * l + dir] = (float*)malloc(sizeof(float) * (long)L * 4 * H);
      gru_fwd(inp[l], L, D, H, W + P->enc[l][dir][0], W + P->enc[l][dir][1], W + P->enc[l][dir][2], dir,
              inp[l + 1] + dir * H, 2 * H, svs[2 * l + dir], tmp);
    }
    D = 2 * H;
  }
  const float* h = inp[nl]; /* (L x A) */
  /* ---- attention forward (oracle attention_fwd) */
  float* Vh = (float*)malloc(sizeof(float) * (long)L * Sc);
  for (int l = 0; l < L; ++l) mv(W + P->V, A, Sc, A, h + (long)l * A, Vh + (long)l * Sc, 0);
  dec_cache C;
  float* cbuf = (float*)malloc(sizeof(float) * (long)T * (Sc + 2 * L + A + S + S + S + S + 1 + M + O + S + A + 3 * S));
  float* p = cbuf;
  C.ws = p; p += (long)T * Sc;
  C.alpha = p; p += (long)T * L;
  float* aprev_all = p; p += (long)T * L;
  C.c = p; p += (long)T * A;
  C.cin = p; p += (long)T * S;
  C.yin = p; p += (long)T * S;
  C.d = p; p += (long)T * S;
  C.sp = p; p += (long)T * S;
  C.ind = p; p += T;
  C.m = p; p += (long)T * M;
  C.logp = p; p += (long)T * O;
  C.v = p; p += (long)T * (S + A);
  C.z = p; p += (long)T * S;
  C.r = p; p += (long)T * S;
  C.hh = p; p += (long)T * S;
  C.am = (int*)malloc(sizeof(int) * (long)T * M);
  float* s = tmp;                  /* S */
  float* th = s + S;               /* Sc */
  float* e = th + Sc;              /* L: uses tmp space beyond; allocate separately below */
  float* eL = (float*)malloc(sizeof(float) * (long)L * 3);
  e = eL;
  float* cs1 = eL + L;
  float* cs2 = eL + 2 * L;
  float* u = (float*)malloc(sizeof(float) * (Mk + 4 * big));
  float* hx = u + Mk;              /* 2S */
  float* o = hx + 2 * big;         /* O */
  float* a2 = o + big;             /* S */
  memset(s, 0, sizeof(float) * S);
  float nll = 0.f;
  for (int t = 0; t < T; ++t) {
    float* ws = C.ws + (long)t * Sc;
    mv(W + P->Ws, S, Sc, S, s, ws, 0);
    for (int j = 0; j < Sc; ++j) ws[j] += W[P->bs + j];
    float emax = -INFINITY;
    for (int l = 0; l < L; ++l) {
      const float* vh = Vh + (long)l * Sc;
      float acc = 0.f;
      for (int j = 0; j < Sc; ++j) acc += W[P->we + j] * tanhf(ws[j] + vh[j]);
      e[l] = acc;
      if (acc > emax) emax = acc;
    }
    float* al = C.alpha + (long)t * L;
    float* ap = aprev_all + (long)t * L;
    float den = 0.f;
    for (int l = 0; l < L; ++l) den += (al[l] = expf(e[l] - emax));
    for (int l = 0; l < L; ++l) al[l] /= den;
    if (t == 0) memset(ap, 0, sizeof(float) * L);
    else memcpy(ap, C.alpha + (long)(t - 1) * L, sizeof(float) * L);
    /* MonotonicAlignment.lua:27-39 */
    float c1 = 0.f, c2 = 0.f, diff = 0.f;
    for (int l = 0; l < L; ++l) {
      c1 += al[l];
      c2 += ap[l];
      diff += c1 - c2;
    }
    (void)cs1; (void)cs2;
    const float pen = c->penalty * (diff > 0.f ? diff : 0.f);
    C.ind[t] = pen > 0.f ? 1.f : 0.f;
    float* cc = C.c + (long)t * A;
    memset(cc, 0, sizeof(float) * A);
    for (int l = 0; l < L; ++l) {
      const float w = al[l];
      const float* hl = h + (long)l * A;
      for (int j = 0; j < A; ++j) cc[j] += w * hl[j];
    }
    float* yin = C.yin + (long)t * S;
    for (int i = 0; i < S; ++i) yin[i] = W[P->by + i] + (t > 0 ? W[P->Wy + (long)i * O + lab[t - 1]] : 0.f);
    float* cin = C.cin + (long)t * S;
    mv(W + P->Wc, A, S, A, cc, cin, 0);
    for (int i = 0; i < S; ++i) cin[i] += W[P->bc + i];
    memcpy(hx, cin, sizeof(float) * S);
    memcpy(hx + S, yin, sizeof(float) * S);
    float* d = C.d + (long)t * S;
    mv(W + P->Wd, 2 * S, S, 2 * S, hx, d, 0);
    for (int i = 0; i < S; ++i) d[i] += W[P->bd + i];
    /* decoder GRU: hx = [s; d] */
    float* sp = C.sp + (long)t * S;
    memcpy(sp, s, sizeof(float) * S);
    memcpy(hx, s, sizeof(float) * S);
    memcpy(hx + S, d, sizeof(float) * S);
    float *z = C.z + (long)t * S, *r = C.r + (long)t * S, *hh = C.hh + (long)t * S;
    mv(W + P->dWz, 2 * S, S, 2 * S, hx, a2, 0);
    for (int i = 0; i < S; ++i) z[i] = sigm(a2[i]);
    mv(W + P->dWr, 2 * S, S, 2 * S, hx, a2, 0);
    for (int i = 0; i < S; ++i) r[i] = sigm(a2[i]);
    for (int i = 0; i < S; ++i) hx[i] = r[i] * s[i];
    mv(W + P->dWh, 2 * S, S, 2 * S, hx, a2, 0);
    for (int i = 0; i < S; ++i) {
      hh[i] = tanhf(a2[i]);
      s[i] = (1.f - z[i]) * s[i] + z[i] * hh[i];
    }
    float* v = C.v + (long)t * (S + A);
    memcpy(v, s, sizeof(float) * S);
    memcpy(v + S, cc, sizeof(float) * A);
    if (mask)
      for (int j = 0; j < S + A; ++j) v[j] *= mask[(long)t * (S + A) + j];
    mv(W + P->Wm, S + A, Mk, S + A, v, u, 0);
    float* mm = C.m + (long)t * M;
    for (int j = 0; j < M; ++j) {
      int best = 0;
      float bv = u[j * k] + W[P->bm + j * k];
      for (int i = 1; i < k; ++i) {
        const float ui = u[j * k + i] + W[P->bm + j * k + i];
        if (ui > bv) { bv = ui; best = i; }
      }
      mm[j] = bv;
      C.am[(long)t * M + j] = best;
    }
    mv(W + P->Wo, M, O, M, mm, o, 0);
    float omax = -INFINITY;
    for (int i = 0; i < O; ++i) {
      o[i] += W[P->bo + i];
      if (o[i] > omax) omax = o[i];
    }
    float se = 0.f;
    for (int i = 0; i < O; ++i) se += expf(o[i] - omax);
    const float lse = omax + logf(se);
    float* lp = C.logp + (long)t * O;
    for (int i = 0; i < O; ++i) lp[i] = o[i] - lse;
    nll -= lp[lab[t]];
  }
  if (normalize) nll /= (float)T;
  /* ---- attention backward (oracle attention_bwd), dlogp = -onehot */
  float* dh = (float*)calloc((size_t)L * A, sizeof(float));
  float* dVh = (float*)calloc((size_t)L * Sc, sizeof(float));
  float* bb = (float*)calloc((size_t)(16 * big + 2 * L + O + Mk + 64), sizeof(float));
  float* ds_carry = bb;            /* S */
  float* ds = ds_carry + big;      /* S */
  float* dc = ds + big;            /* A */
  float* dv = dc + big;            /* S + A */
  float* dsp = dv + big;           /* S */
  float* dd = dsp + big;           /* S */
  float* dcy = dd + big;           /* 2S */
  float* tv = dcy + 2 * big;       /* 2S */
  float* dws = tv + 2 * big;       /* Sc */
  float* gz = dws + big;           /* S: daz / dah / dar */
  float* dalpha = gz + 3 * big;    /* L */
  float* dacarry = dalpha + L;     /* L */
  float* dO = dacarry + L;         /* O */
  float* du = dO + O;              /* Mk */
  for (int t = T - 1; t >= 0; --t) {
    const float* lp = C.logp + (long)t * O;
    for (int i = 0; i < O; ++i) dO[i] = expf(lp[i]) - (i == lab[t] ? 1.f : 0.f);
    ger(G + P->Wo, M, O, M, scale, dO, C.m + (long)t * M);
    for (int i = 0; i < O; ++i) G[P->bo + i] += scale * dO[i];
    memset(du, 0, sizeof(float) * Mk);
    for (int j = 0; j < M; ++j) {
      float dm = 0.f;
      for (int i = 0; i < O; ++i) dm += W[P->Wo + (long)i * M + j] * dO[i];
      du[j * k + C.am[(long)t * M + j]] = dm;
    }
    const float* v = C.v + (long)t * (S + A);
    ger(G + P->Wm, S + A, Mk, S + A, scale, du, v);
    for (int i = 0; i < Mk; ++i) G[P->bm + i] += scale * du[i];
    memset(dv, 0, sizeof(float) * (S + A));
    mtv(W + P->Wm, S + A, Mk, S + A, du, dv);
    if (mask)
      for (int j = 0; j < S + A; ++j) dv[j] *= mask[(long)t * (S + A) + j];
    for (int i = 0; i < S; ++i) ds[i] = dv[i] + ds_carry[i];
    memcpy(dc, dv + S, sizeof(float) * A);
    const float *sp = C.sp + (long)t * S, *d = C.d + (long)t * S;
    const float *z = C.z + (long)t * S, *r = C.r + (long)t * S, *hh = C.hh + (long)t * S;
    /* oracle _gru_dec_bwd */
    float *daz = gz, *dah = gz + big, *dar = gz + 2 * big;
    for (int i = 0; i < S; ++i) {
      const float dz = ds[i] * (hh[i] - sp[i]);
      dah[i] = ds[i] * z[i] * (1.f - hh[i] * hh[i]);
      dsp[i] = ds[i] * (1.f - z[i]);
      daz[i] = dz * z[i] * (1.f - z[i]);
    }
    for (int i = 0; i < S; ++i) tv[i] = r[i] * sp[i];
    memcpy(tv + S, d, sizeof(float) * S);
    ger(G + P->dWh, 2 * S, S, 2 * S, scale, dah, tv);
    memset(dcy, 0, sizeof(float) * 2 * S);
    mtv(W + P->dWh, 2 * S, S, 2 * S, dah, dcy); /* drhx */
    memcpy(dd, dcy + S, sizeof(float) * S);
    for (int i = 0; i < S; ++i) {
      const float dr = dcy[i] * sp[i];
      dsp[i] += dcy[i] * r[i];
      dar[i] = dr * r[i] * (1.f - r[i]);
    }
    memcpy(tv, sp, sizeof(float) * S);
    ger(G + P->dWz, 2 * S, S, 2 * S, scale, daz, tv);
    ger(G + P->dWr, 2 * S, S, 2 * S, scale, dar, tv);
    memset(dcy, 0, sizeof(float) * 2 * S);
    mtv(W + P->dWz, 2 * S, S, 2 * S, daz, dcy);
    mtv(W + P->dWr, 2 * S, S, 2 * S, dar, dcy);
    for (int i = 0; i < S; ++i) {
      dsp[i] += dcy[i];
      dd[i] += dcy[S + i];
    }
    /* d = Wd [c_in; y_in] + bd */
    memcpy(tv, C.cin + (long)t * S, sizeof(float) * S);
    memcpy(tv + S, C.yin + (long)t * S, sizeof(float) * S);
    ger(G + P->Wd, 2 * S, S, 2 * S, scale, dd, tv);
    for (int i = 0; i < S; ++i) G[P->bd + i] += scale * dd[i];
    memset(dcy, 0, sizeof(float) * 2 * S);
    mtv(W + P->Wd, 2 * S, S, 2 * S, dd, dcy); /* dcin | dyin */
    const float* cc = C.c + (long)t * A;
    ger(G + P->Wc, A, S, A, scale, dcy, cc);
    for (int i = 0; i < S; ++i) G[P->bc + i] += scale * dcy[i];
    mtv(W + P->Wc, A, S, A, dcy, dc);
    for (int i = 0; i < S; ++i) {
      if (t > 0) G[P->Wy + (long)i * O + lab[t - 1]] += scale * dcy[S + i];
      G[P->by + i] += scale * dcy[S + i];
    }
    /* c = alpha^T h; MonotonicAlignment backward; softmax backward */
    const float* al = C.alpha + (long)t * L;
    float sad = 0.f;
    for (int l = 0; l < L; ++l) {
      const float* hl = h + (long)l * A;
      float acc = 0.f;
      for (int j = 0; j < A; ++j) acc += dc[j] * hl[j];
      float* dhl = dh + (long)l * A;
      for (int j = 0; j < A; ++j) dhl[j] += al[l] * dc[j];
      const float gdiff = c->penalty * (float)(L - l) * C.ind[t];
      dalpha[l] = acc + dacarry[l] + gdiff;
      dacarry[l] = -gdiff;
      sad += al[l] * dalpha[l];
    }
    const float* ws = C.ws + (long)t * Sc;
    memset(dws, 0, sizeof(float) * Sc);
    for (int l = 0; l < L; ++l) {
      const float de = al[l] * (dalpha[l] - sad);
      const float* vh = Vh + (long)l * Sc;
      float* dz = dVh + (long)l * Sc;
      for (int j = 0; j < Sc; ++j) {
        const float tj = tanhf(ws[j] + vh[j]);
        G[P->we + j] += scale * de * tj;
        const float g = de * W[P->we + j] * (1.f - tj * tj);
        dz[j] += g;
        dws[j] += g;
      }
    }
    ger(G + P->Ws, S, Sc, S, scale, dws, sp);
    for (int j = 0; j < Sc; ++j) G[P->bs + j] += scale * dws[j];
    memcpy(ds_carry, dsp, sizeof(float) * S);
    mtv(W + P->Ws, S, Sc, S, dws, ds_carry);
  }
  /* Vh = h V^T */
  for (int l = 0; l < L; ++l) {
    ger(G + P->V, A, Sc, A, scale, dVh + (long)l * Sc, h + (long)l * A);
    mtv(W + P->V, A, Sc, A, dVh + (long)l * Sc, dh + (long)l * A);
  }
  /* ---- encoder backward (oracle encoder_bwd) */
  float* dcur = dh;
  for (int l = nl - 1; l >= 0; --l) {
    const int H = l == nl - 1 ? c->Ho : c->Hh;
    const int Dl = l == 0 ? c->F : 2 * c->Hh;
    float* dx = (float*)calloc((size_t)L * Dl, sizeof(float));
    for (int dir = 0; dir < 2; ++dir)
      gru_bwd(inp[l], L, Dl, H, W + P->enc[l][dir][0], W + P->enc[l][dir][1], W + P->enc[l][dir][2], dir,
              svs[2 * l + dir], dcur + dir * H, 2 * H, dx, G + P->enc[l][dir][0], G + P->enc[l][dir][1],
              G + P->enc[l][dir][2], scale, tmp);
    free(dcur);
    dcur = dx;
  }
  free(dcur);
  for (int l = 0; l < nl; ++l) {
    free(inp[l + 1]);
    free(svs[2 * l]);
    free(svs[2 * l + 1]);
  }
  free(inp); free(svs); free(tmp); free(Vh); free(cbuf); free(C.am); free(eL); free(u); free(dVh); free(bb);
  return nll;
}

/* The minibatch (timit/timit.lua:240-295): B utterances x (B, L, F), labels (B, T), each forwarded and
 * back-propagated alone, grads (flat, overwritten) = (1/B if B > 1) * sum of the utterances' gradients, nll[b]
 * per utterance.  masks: (B, T, S + A) nn.Dropout multipliers or NULL.  threads: OpenMP threads (<= 0: all).
 * Each thread accumulates into its own gradient buffer; the buffers are summed in thread order. */
int s2s_cpu_step(const s2s_cpu_cfg* c, const float* params, const float* x, const int* labels, int B, int L, int T,
                 const float* masks, int normalize, int threads, float* grads, float* nll) {
  const layout P = layout_of(c);
  const float scale = B > 1 ? 1.f / (float)B : 1.f;
  int nt = 1;
#ifdef _OPENMP
  nt = threads > 0 ? threads : omp_get_max_threads();
#endif
  if (nt > B) nt = B;
  float* part = (float*)calloc((size_t)nt * P.total, sizeof(float));
  if (!part) return 1;
  const int A = 2 * c->Ho, S = c->S;
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1)
  for (int b = 0; b < B; ++b) {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    nll[b] = utterance(c, &P, params, x + (long)b * L * c->F, labels + (long)b * T, L, T,
                       masks ? masks + (long)b * T * (S + A) : NULL, normalize, part + (long)tid * P.total, scale);
  }
  memset(grads, 0, sizeof(float) * P.total);
  for (int i = 0; i < nt; ++i) {
    const float* q = part + (long)i * P.total;
    for (long j = 0; j < P.total; ++j) grads[j] += q[j];
  }
  free(part);
  return 0;
}
