// Host sanitizer run of the oracle (SURVEY 5 "Race detection / sanitizers": -fsanitize=address,
// undefined on the oracle).  Test infrastructure only: `make -C oracle sanitize` builds this file with
// oracle.cpp under ASan + UBSan (no recovery), tests/test_sanitizers.py runs it.  It drives every
// exported entry point on small cases, including the edge cases the GPU tests cover (a ray with
// all-zero weights, one sample pair, 512 samples, masked rays), in fp64 and fp32, single-threaded.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

struct orc_spec { int32_t D, W, Dc, Wc, skip, min_deg, max_deg, deg_view; };
struct orc_step_args {
  int32_t n, num_levels; const int32_t* S; int32_t randomized, white;
  float padding, coarse_mult, loss_mult_sum;
  uint64_t seed; uint32_t step, ray_base;
  const float *o, *d, *radius, *near_, *far_, *lossmult, *pix;
  const float* const* t_override;
  const uint8_t* const* relu_mask;
  float* const* t_out; void* const* w_out; void* const* C_out; void* const* sigma_out; void* const* rgb_out;
  void* const* dsigma_out; void* const* drgb_out; void* grads; void* loss;
  int32_t nthreads;
  int64_t* mask_flips;
  int32_t lindisp, ray_shape;
  float density_bias, rgb_padding;
};
extern "C" {
int64_t orc_param_count(const orc_spec* s);
void orc_layer_sizes(const orc_spec* s, int32_t* out);
void orc_sample_stratified(int32_t n, int32_t S, const float* nears, const float* fars, int32_t randomized,
                           uint64_t seed, uint32_t step, uint32_t level, uint32_t ray_base, float* t, int32_t lindisp);
void orc_sample_pdf(int32_t n, int32_t S_in, const float* t_in, const float* w, int32_t S_out, float padding,
                    int32_t randomized, uint64_t seed, uint32_t step, uint32_t level, uint32_t ray_base,
                    float* t_out, int32_t* idx);
void orc_step_f64(const orc_spec* s, const float* P, const orc_step_args* a);
void orc_step_f32(const orc_spec* s, const float* P, const orc_step_args* a);
void orc_adam_step(int64_t n, float* p, const float* g, float* m, float* v, float lr, int32_t iteration);
float orc_lr_decay(int32_t step, float init, float fin, int32_t max_steps, int32_t delay_steps, float delay_mult);
void orc_glorot_init(const orc_spec* s, uint64_t seed, float* P);
}

static int fails = 0;
static void check(bool ok, const char* what) {
  if (!ok) { std::fprintf(stderr, "FAIL: %s\n", what); ++fails; }
}
template <class T>
static bool finite(const std::vector<T>& v) {
  for (T x : v) if (!std::isfinite((double)x)) return false;
  return true;
}

template <class T>
static void run_step(const orc_spec& sp, int n, int S0, int S1, bool masked, bool f64, int lindisp = 0,
                     int ray_shape = 0) {
  const int64_t P = orc_param_count(&sp);
  std::vector<float> params(P);
  orc_glorot_init(&sp, 7, params.data());
  std::vector<float> o(3 * n), d(3 * n), r(n), nr(n, 2.0f), fr(n, 6.0f), lm(n, 1.0f), pix(3 * n);
  for (int i = 0; i < n; ++i) {
    o[3 * i] = 0.1f * i; o[3 * i + 1] = -0.2f; o[3 * i + 2] = 4.0f;
    d[3 * i] = 0.05f * (i % 3); d[3 * i + 1] = 0.02f; d[3 * i + 2] = -1.0f;
    r[i] = 0.0012f;
    pix[3 * i] = 0.3f; pix[3 * i + 1] = 0.6f; pix[3 * i + 2] = 0.9f;
  }
  if (masked) lm[0] = 0.0f;
  float msum = 0.0f;
  for (float x : lm) msum += x;
  const int32_t S[2] = {S0, S1};
  std::vector<float> t0((size_t)n * (S0 + 1)), t1((size_t)n * (S1 + 1));
  std::vector<T> w0((size_t)n * S0), w1((size_t)n * S1), C0(3 * n), C1(3 * n), s0((size_t)n * S0), s1((size_t)n * S1),
      rgb0((size_t)3 * n * S0), rgb1((size_t)3 * n * S1), ds0((size_t)n * S0), ds1((size_t)n * S1),
      dr0((size_t)3 * n * S0), dr1((size_t)3 * n * S1), G(P);
  T loss = 0;
  float* t_out[2] = {t0.data(), t1.data()};
  void* w_out[2] = {w0.data(), w1.data()};
  void* C_out[2] = {C0.data(), C1.data()};
  void* s_out[2] = {s0.data(), s1.data()};
  void* rgb_out[2] = {rgb0.data(), rgb1.data()};
  void* ds_out[2] = {ds0.data(), ds1.data()};
  void* dr_out[2] = {dr0.data(), dr1.data()};
  int64_t flips[2] = {0, 0};  // per level
  orc_step_args a{n, 2, S, 1, 1, 0.01f, 0.1f, msum, 42, 3, 5, o.data(), d.data(), r.data(), nr.data(), fr.data(),
                  lm.data(), pix.data(), nullptr, nullptr, t_out, w_out, C_out, s_out, rgb_out, ds_out, dr_out,
                  G.data(), &loss, 1, flips, lindisp, ray_shape, -1.0f, 0.001f};
  if (f64) orc_step_f64(&sp, params.data(), &a);
  else orc_step_f32(&sp, params.data(), &a);
  check(finite(G) && finite(C1) && finite(ds1) && finite(dr0) && std::isfinite((double)loss), "step outputs finite");
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < S1; ++k) check(t1[(size_t)i * (S1 + 1) + k] <= t1[(size_t)i * (S1 + 1) + k + 1], "t sorted");
  if (masked) {
    bool zero = true;
    for (int k = 0; k < S1; ++k) zero = zero && ds1[k] == 0 && dr1[3 * k] == 0;
    check(zero, "masked ray has zero output gradients");
  }
  // Adam on the gradient (float view)
  std::vector<float> g(P), m(P, 0.0f), v(P, 0.0f);
  for (int64_t i = 0; i < P; ++i) g[i] = (float)G[i];
  orc_adam_step(P, params.data(), g.data(), m.data(), v.data(), orc_lr_decay(3, 5e-4f, 5e-6f, 1000000, 2500, 0.01f), 3);
  check(finite(params), "Adam output finite");
}

int main() {
  const orc_spec ref{8, 256, 1, 128, 4, 0, 16, 4}, small{4, 128, 1, 128, 4, 0, 16, 4};
  std::vector<int32_t> sizes(2 * 11);
  orc_layer_sizes(&ref, sizes.data());
  check(sizes[0] == 96 * 256 && orc_param_count(&ref) == 546948, "reference layer sizes");
  run_step<double>(ref, 3, 64, 64, false, true);
  run_step<double>(ref, 2, 64, 128, true, true);
  run_step<float>(ref, 3, 128, 64, false, false);
  run_step<float>(small, 4, 64, 64, true, false);
  run_step<double>(ref, 1, 512, 512, false, true);
  run_step<double>(ref, 2, 64, 64, false, true, 1, 1);  // LinDisp sampling, cylindrical Gaussians
  // the resampler on a ray with all-zero weights (uniform pdf after padding) and on one sample pair
  std::vector<float> tin = {2.0f, 3.0f, 4.0f, 5.0f, 6.0f}, w(4, 0.0f), tout(9);
  std::vector<int32_t> idx(9);
  orc_sample_pdf(1, 4, tin.data(), w.data(), 8, 0.01f, 1, 9, 1, 1, 0, tout.data(), idx.data());
  for (int k = 0; k < 9; ++k) check(idx[k] >= 0 && idx[k] < 4 && std::isfinite(tout[k]), "pdf on zero weights");
  std::vector<float> t1(3), nears{2.0f}, fars{6.0f};
  orc_sample_stratified(1, 2, nears.data(), fars.data(), 1, 5, 2, 0, 0, t1.data(), 0);
  check(t1[0] <= t1[1] && t1[1] <= t1[2], "stratified S=2");
  std::printf("oracle sanitizer run: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
