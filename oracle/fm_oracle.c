/*
 * CPU oracle — TEST INFRASTRUCTURE ONLY (checker and bench.py cpu_baseline "port").
 *
 * Plain-C fp64 restatement of one mini-batch SGD iteration of Rainbowboys/fm_spark
 * (FactorizationMachinesSGD.scala:116-211 over the plan of
 * FactorizationMachinesModel.scala:135-234), eager like the reference: the L1
 * soft-threshold is applied to every present row every iteration (SGD.scala:157-181).
 * Same math as oracle/fm_ref.py; the product path never links this file.
 *
 * Parallelism (OpenMP): forward over samples; per-feature gradient sums with
 * owner-computes (thread t sums ids with id % T == t, scanning entries in CSR order), so
 * the result is bitwise independent of the thread count; update + L1 over rows.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct oracle_model {
  int64_t F;
  int32_t k;
  double w0;
  double* w;        /* [F] */
  double* V;        /* [F*k] */
  uint8_t* present; /* [F] */
  double* GW;       /* [F] scratch */
  double* GV;       /* [F*k] scratch */
  uint8_t* touched; /* [F] scratch */
  double* S;        /* [cap_rows*k] per-sample vfxiSum */
  double* yhat;     /* [cap_rows] */
  int64_t cap_rows;
} oracle_model;

int oracle_create(int64_t F, int32_t k, double w0, oracle_model** out) {
  oracle_model* m = (oracle_model*)calloc(1, sizeof(oracle_model));
  if (!m) return -2;
  m->F = F;
  m->k = k;
  m->w0 = w0;
  m->w = (double*)calloc((size_t)F, sizeof(double));
  m->V = (double*)calloc((size_t)F * k, sizeof(double));
  m->present = (uint8_t*)calloc((size_t)F, 1);
  m->GW = (double*)calloc((size_t)F, sizeof(double));
  m->GV = (double*)calloc((size_t)F * k, sizeof(double));
  m->touched = (uint8_t*)calloc((size_t)F, 1);
  if (!m->w || !m->V || !m->present || !m->GW || !m->GV || !m->touched) return -2;
  *out = m;
  return 0;
}

void oracle_destroy(oracle_model* m) {
  if (!m) return;
  free(m->w); free(m->V); free(m->present); free(m->GW); free(m->GV); free(m->touched);
  free(m->S); free(m->yhat);
  free(m);
}

void oracle_load(oracle_model* m, const int32_t* ids, int64_t n, const double* w, const double* V) {
  for (int64_t i = 0; i < n; ++i) {
    int64_t id = ids[i];
    m->w[id] = w[i];
    memcpy(m->V + id * m->k, V + i * m->k, sizeof(double) * m->k);
    m->present[id] = 1;
  }
}

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* Marks [b, e) present with N(0, sd^2) values (baseline timing only; not the device draw). */
void oracle_init_random(oracle_model* m, uint64_t seed, double sd, int64_t b, int64_t e) {
  const int32_t k = m->k;
#pragma omp parallel for schedule(static)
  for (int64_t id = b; id < e; ++id) {
    for (int32_t f = -1; f < k; ++f) {
      uint64_t h1 = splitmix64(seed ^ splitmix64((uint64_t)id * 131 + (uint64_t)(f + 1)));
      uint64_t h2 = splitmix64(h1);
      double u1 = ((h1 >> 11) + 1) * (1.0 / 9007199254740993.0);
      double u2 = (h2 >> 11) * (1.0 / 9007199254740992.0);
      double g = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2) * sd;
      if (f < 0) m->w[id] = g; else m->V[id * k + f] = g;
    }
    m->present[id] = 1;
  }
}

/* Marks [b, e) present with the device's createInitialModel draw (fm_kernels.hip gauss_draw:
 * N(0, sd^2) keyed by (seed, id, factor; -1 = w), Box-Muller in fp64, rounded to fp32 as the
 * device table holds it), so a whole-table comparison starts from the same table. */
static inline double device_gauss(uint64_t seed, int64_t id, int f, double sd) {
  const uint64_t c = ((uint64_t)id << 10) ^ (uint64_t)(f + 1);
  const uint64_t h1 = splitmix64(seed ^ splitmix64(c));
  const uint64_t h2 = splitmix64(h1 ^ 0x632BE59BD9B4E019ull);
  const double u1 = (double)((h1 >> 11) + 1) * 0x1.0p-53;
  const double u2 = (double)(h2 >> 11) * 0x1.0p-53;
  const double g = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
  return (double)(float)(g * sd);
}

void oracle_init_device_draw(oracle_model* m, uint64_t seed, double sd, int64_t b, int64_t e) {
  const int32_t k = m->k;
#pragma omp parallel for schedule(static)
  for (int64_t id = b; id < e; ++id) {
    m->w[id] = device_gauss(seed, id, -1, sd);
    for (int32_t f = 0; f < k; ++f) m->V[id * k + f] = device_gauss(seed, id, f, sd);
    m->present[id] = 1;
  }
}

static void ensure_rows(oracle_model* m, int64_t B) {
  if (B <= m->cap_rows) return;
  free(m->S); free(m->yhat);
  m->S = (double*)malloc(sizeof(double) * (size_t)B * m->k);
  m->yhat = (double*)malloc(sizeof(double) * (size_t)B);
  m->cap_rows = B;
}

/* One iteration.  Returns 1 (nothing done) when n_rows == 0 (SGD.scala:126-128). */
int oracle_step(oracle_model* m, const int64_t* row_ptr, const int32_t* col, const double* val,
                const double* label, int64_t n_rows, int32_t t, double step_size, double reg_param,
                double* loss_out, int64_t* n_loss_out, int64_t* n_unique_out) {
  if (n_rows == 0) return 1;
  const int32_t k = m->k;
  const double eta = step_size / sqrt((double)t);          /* SGD.scala:121 */
  const double lam = eta * reg_param;                       /* SGD.scala:122 */
  const double mdb = (double)n_rows;                        /* miniBatchSize, SGD.scala:124 */
  ensure_rows(m, n_rows);
  double loss = 0.0;
  int64_t n_loss = 0;
  /* forward, Model.scala:173-221 */
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : loss, n_loss)
  for (int64_t s = 0; s < n_rows; ++s) {
    double* S = m->S + s * k;
    for (int32_t f = 0; f < k; ++f) S[f] = 0.0;
    double wsum = 0.0, vv = 0.0;
    const int64_t e0 = row_ptr[s], e1 = row_ptr[s + 1];
    for (int64_t e = e0; e < e1; ++e) {
      const int64_t id = col[e];
      const double x = val[e];
      const double* v = m->V + id * k;
      wsum += m->w[id] * x;                                  /* wixi  :178 */
      double v2 = 0.0;
      for (int32_t f = 0; f < k; ++f) {
        S[f] += v[f] * x;                                    /* VectorSum(vfxi) :191 */
        v2 += v[f] * v[f];
      }
      vv += v2 * x * x;                                      /* vi2xi2 :256-258 */
    }
    double ss = 0.0;
    for (int32_t f = 0; f < k; ++f) ss += S[f] * S[f];
    const double yhat = 0.5 * (ss - vv) + wsum + m->w0;      /* :221, sumVx :260-262 */
    m->yhat[s] = yhat;
    if (e1 > e0) {
      const double d = yhat - label[s];
      loss += d * d;                                         /* :230, SGD.scala:134-138 */
      n_loss += 1;
    }
  }
  /* per-feature gradient sums, SGD.scala:142-155 (owner-computes, CSR order) */
  int64_t n_unique = 0;
#pragma omp parallel reduction(+ : n_unique)
  {
    int T = 1, me = 0;
#ifdef _OPENMP
    T = omp_get_num_threads();
    me = omp_get_thread_num();
#endif
    for (int64_t s = 0; s < n_rows; ++s) {
      const int64_t e0 = row_ptr[s], e1 = row_ptr[s + 1];
      if (e0 == e1) continue;
      const double yhat = m->yhat[s], y = label[s], r = yhat - y;
      const double* S = m->S + s * k;
      for (int64_t e = e0; e < e1; ++e) {
        const int64_t id = col[e];
        if ((int)(id % T) != me) continue;
        const double x = val[e];
        const double* v = m->V + id * k;
        double* gv = m->GV + id * k;
        if (!m->touched[id]) {
          m->touched[id] = 1;
          n_unique += 1;
        }
        m->GW[id] += x * yhat - y;                           /* P1: deltaWi*pred - label */
        for (int32_t f = 0; f < k; ++f) gv[f] += (S[f] * x - (v[f] * x) * x) * r;
      }
    }
  }
  /* update + L1 over every present (or touched) row, SGD.scala:157-181 */
  const double scale_v = eta / mdb;
#pragma omp parallel for schedule(static)
  for (int64_t id = 0; id < m->F; ++id) {
    if (!m->present[id] && !m->touched[id]) continue;
    double* v = m->V + id * k;
    double wn = m->w[id];
    if (m->touched[id]) {
      wn = wn - (m->GW[id] / mdb) * eta;
      double* gv = m->GV + id * k;
      for (int32_t f = 0; f < k; ++f) {
        v[f] = v[f] - gv[f] * scale_v;
        gv[f] = 0.0;
      }
      m->GW[id] = 0.0;
      m->touched[id] = 0;
      m->present[id] = 1;
    }
    {
      double a = fabs(wn) - lam;
      m->w[id] = a > 0.0 ? copysign(a, wn) : 0.0 * wn;
    }
    for (int32_t f = 0; f < k; ++f) {
      double a = fabs(v[f]) - lam;
      v[f] = a > 0.0 ? copysign(a, v[f]) : 0.0 * v[f];
    }
  }
  if (loss_out) *loss_out = loss;
  if (n_loss_out) *n_loss_out = n_loss;
  if (n_unique_out) *n_unique_out = n_unique;
  return 0;
}

double* oracle_w(oracle_model* m) { return m->w; }
double* oracle_V(oracle_model* m) { return m->V; }
uint8_t* oracle_present(oracle_model* m) { return m->present; }

int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void oracle_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}
