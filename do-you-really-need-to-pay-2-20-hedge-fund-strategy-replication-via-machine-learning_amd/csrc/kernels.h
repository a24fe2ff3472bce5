// Host-side launcher declarations of the hfrep gfx950 kernel library.
// Kernel translation units (*.hip) define these; bindings.cpp exposes them as torch ops.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hfrep {

// storage dtype codes shared by all launchers
enum DType : int { DT_F32 = 0, DT_BF16 = 1 };

// ---- lstm.hip (return false if H is not an instantiated hidden size) ----
bool launch_lstm_fwd(int dt, const void* zx, const float* U, void* hs, void* gates, void* cs, int B, int Tn, int H,
                     int act, hipStream_t s);
bool launch_lstm_bwd(int dt, const void* dH, const void* gates, const void* cs, const float* U, void* dZ, int B,
                     int Tn, int H, int act, hipStream_t s);
bool launch_lstm_tfwd(int dt, const void* dzx, const void* gates, const void* cs, const float* U, void* hds,
                      void* zds, void* cds, int B, int Tn, int H, int act, hipStream_t s);
bool launch_lstm_tbwd(int dt, const void* dH, const void* dHd, const void* gates, const void* cs, const void* zds,
                      const void* cds, const float* U, void* dZ, void* dZd, int B, int Tn, int H, int act,
                      hipStream_t s);

// ---- lstm2.hip (bf16, fused input projection, blocked tapes; H == 100, K <= 128) ----
size_t lstm2_tape_elems(int B, int Tn);
bool lstm2_supported(int H, int K);
void launch_lstm2_fwd(const void* x, const float* W, const float* b, const float* U, void* hs, void* tape, int B, int Tn,
                      int K, int H, int act, hipStream_t s);
void launch_lstm2_tfwd(const void* xd, const float* W, const float* U, const void* tape, void* hds, void* ttape, int B,
                       int Tn, int K, int H, int act, hipStream_t s);
// W / dX non-null: the input gradient dX = dZ W^T (K columns) is produced by the same launch
// head_d / head_dd + hw: dH (dHdot) = d[b] * hw[t H + h] generated in-kernel (Flatten -> Dense(1) head
// adjoint); otherwise dH / dHd tensors (nullptr = zeros)
void launch_lstm2_bwd(const void* dH, const void* tape, const float* U, void* dZ, const float* W, void* dX, int K,
                      int B, int Tn, int H, int act, hipStream_t s, const void* head_d = nullptr,
                      const float* hw = nullptr);
void launch_lstm2_tbwd(const void* dH, const void* dHd, const void* tape, const void* ttape, const float* U, void* dZ,
                       void* dZd, const float* W, void* dX, void* dXd, int K, int B, int Tn, int H, int act,
                       hipStream_t s, const void* head_d = nullptr, const void* head_dd = nullptr,
                       const float* hw = nullptr);

// ---- lstm_f32.hip (fp32, fused input projection, exact-fp32 MFMA; H == 100, K in {32, 35, 36, 100},
//      act in {linear, sigmoid, tanh}; false = not supported).  Tapes: lane-native blocked fp32
//      (lstmf_tape_elems floats; primal = gate activations + c, tangent = zdot + cdot). ----
bool lstmf_supported(int H, int K, int act);
size_t lstmf_tape_elems(int B, int Tn);
bool launch_lstmf_fwd(const float* x, const float* W, const float* b, const float* U, float* hs, float* tape, int B,
                      int Tn, int K, int H, int act, hipStream_t s);
bool launch_lstmf_tfwd(const float* xd, const float* W, const float* U, const float* tape, float* hds, float* ttape,
                       int B, int Tn, int K, int H, int act, hipStream_t s);
// BPTT / tangent reverse on those tapes (dH / dHd may be null = zeros); dZ / dZd row-major (B,T,4H)
// hd / hw (HEAD): dH = hd (x) hw generated in the kernel (the critic head's adjoint: hd (B), hw (Tn H));
// dH is then unused.  Not with the exact-fp32 BPTT (lstmf_head_supported() false: materialise dH).
bool launch_lstmf_bwd(const float* dH, const float* tape, const float* U, float* dZ, int B, int Tn, int H, int act,
                      hipStream_t s, const float* hd = nullptr, const float* hw = nullptr);
bool lstmf_head_supported();
// hw (HEAD): dH = hd (x) hw, dHd = hdd (x) hw generated in the kernel (a null factor: that adjoint is 0)
bool launch_lstmf_tbwd(const float* dH, const float* dHd, const float* tape, const float* ttape, const float* U, float* dZ,
                       float* dZd, int B, int Tn, int H, int act, hipStream_t s, const float* hd = nullptr,
                       const float* hdd = nullptr, const float* hw = nullptr);
// fused fp32 LSTM weight gradients (K in {32, 36, 100}, H = 100, N = 400): gW += X^T dZ (+ Xd^T dZd),
// gU += Hprev^T dZ (+ Hdprev^T dZd), gb += colsum dZ, through per-workgroup slabs in ws
// (lstmf_wgrad_workspace_floats) and one fixed-order reduce
bool lstmf_wgrad_supported(int K, int H, int N);
// impl: 0 = default (exact under HFREP_FP32_EXACT=1, else the pair split for K <= 36 and the quad split for K = 100), 1 = exact-fp32
// MFMA, 2 = the three-term bf16 split (pair), 3 = the three-term bf16 split (quad)
size_t lstmf_wgrad_workspace_floats(int M, int K, int impl = 0);
bool launch_lstmf_wgrad(const void* X, const void* Hs, const void* D, const void* Xd, const void* Hds, const void* Dd,
                        float* gW, float* gU, float* gb, int M, int K, int Tn, float* ws, hipStream_t s, int impl = 0,
                        int pm = 0);  // pm: FP3-plane operands (bit 1 X, 2 H, 4 D interleaved)
// fp32 input gradient X (M, KO) = D (M, N) W^T, W (KO, N) row-major; N = 400, KO <= 112
bool lstmf_dgrad_supported(int N, int KO);
// forward kernel selection: 1 = exact-fp32 everywhere, 2 = split recurrent product for K <= 36 (default);
// returns the previous setting
int set_lstmf_fwd_impl(int v);  // 1: exact-fp32 forward everywhere, 2: the split-recurrent one for K <= 36
int set_lstmf_bwd_impl(int v);  // 2: the exact-fp32 BPTT kernel, 3: the split-recurrent one
// impl: 0 = default (exact under HFREP_FP32_EXACT=1, else the LDS-staged split for KO > 64), 1 = exact, 3 = three-term bf16 split
bool launch_lstmf_dgrad(const void* D, const float* W, float* X, int M, int N, int KO, hipStream_t s, int impl = 0,
                        bool pd = false);  // pd: dZ as FP3 planes (interleaved gate order)
// FP3 planes (csrc/lstm_f32.hip): fp32 (M, C) <-> bf16 (M, 3, C) exact split planes; interleave: C = 400 in
// the gate-interleaved column order k = 4 u + q
void launch_fp3_split(const float* x, uint16_t* p, int64_t M, int C, bool interleave, hipStream_t s);
void launch_fp3_join(const uint16_t* p, float* x, int64_t M, int C, bool interleave, hipStream_t s);

// ---- ae.hip (factor autoencoder: the whole Keras fit -- MSE, Nadam, EarlyStopping -- in one launch) ----
bool ae_fit_supported(int A, int k, int batch);
// one independent fit: its data, batch orders (epochs, nt), weights (A x k), Nadam slots and shared
// counters, and the per-epoch (loss, val_loss) history + epochs-run outputs
struct AeFitJob {
  const float* Xt;
  const float* Xv;
  const int* order;
  float *We, *Wd, *mWe, *vWe, *mWd, *vWd, *step, *m_cache;
  double* hist;
  int* nep;
  int nt, nv, epochs, patience, k, pad_;
};
// `jobs` is a device array of njobs records (one workgroup each)
void launch_ae_fit(bool bf16, const AeFitJob* jobs, int njobs, int batch, float lr, float b1, float b2, float eps, int A,
                   hipStream_t s);

// ---- gemm.hip ----
// C[M,N] = act(A[M,K] . op(W) + bias);  op(W) = W (K,N) or W^T when w_trans (W stored (N,K)).
// A and C share the activation dtype `dt`; W and bias are fp32 (converted while staging).
void launch_linear(int dt, const void* A, const float* W, const float* bias, void* C, int M, int N, int K,
                   int w_trans, int act, hipStream_t s);
// gW[K,N] += sum_m X[m,:]^T D[m,:]  (and gb[N] += sum_m D[m,:] when gb != nullptr).
// shiftT > 0: X row m is replaced by row m-1, and by zeros where m % shiftT == 0 (h_{t-1} trick).
// Uses split-M fp32 slabs in `ws` (size >= wgrad_workspace_floats) and a reduce launch.
// HFREP_FP32_EXACT=1: fp32 products on the exact-fp32 MFMA instead of the three-term bf16 split
bool fp32_exact_mode();
size_t wgrad_workspace_floats(int M, int K, int N);
void launch_wgrad(int dt, const void* X, const void* D, float* gW, float* gb, int M, int K, int N, int shiftT,
                  float* ws, hipStream_t s);

// ---- gemm2.hip (bf16) ----
size_t lstm_wgrad2_workspace_floats(int M, int K, int Hd, int N);
void launch_lstm_wgrad2(const void* X0, const void* H0, const void* D0, const void* X1, const void* H1, const void* D1,
                        float* gW, float* gU, float* gb, int M, int K, int Hd, int N, int Tn, float* ws, hipStream_t s);
// split-slab reduce shared by wgrad2 / wgrad3 / the fp32 kernels: slab rows 0..K-1 -> gW, Ks..Ks+Hd-1 -> gU,
// Ks+Hd -> gb (if non-null); Ks (default K) > K: rows K..Ks-1 are image padding (K = 35 in a 36-row image)
void launch_lstm_wgrad2_reduce(const float* ws, float* gW, float* gU, float* gb, int splits, int K, int Hd, int N,
                               hipStream_t s, int Ks = 0);
void launch_linear2(const void* A, const float* W, const float* bias, void* C, int M, int N, int K, int w_trans, int act,
                    hipStream_t s);

// ---- wgrad3.hip (bf16 LDS-DMA streaming LSTM wgrad; Hd == 100, K in {32, 100}; false = use wgrad2) ----
bool lstm_wgrad3_supported(int M, int K, int Hd, int N);
size_t lstm_wgrad3_workspace_floats(int K, int Hd, int N);
bool launch_lstm_wgrad3(const void* X0, const void* H0, const void* D0, const void* X1, const void* H1, const void* D1,
                        float* gW, float* gU, float* gb, int M, int K, int Hd, int N, int Tn, float* ws, hipStream_t s);

// ---- skinny.hip (bf16 / fp32, N <= 4 output columns, K % 8 == 0: the Flatten -> Dense(1) critic head) ----
bool skinny_supported(int K, int N);
bool narrow_supported(int K, int N);  // 4 < N <= 64, K <= 128 even (bf16 forward only)
void launch_narrow_fwd(const void* x, const float* W, const float* b, void* y, int M, int K, int N, int act,
                       hipStream_t s);
// exact-fp32 narrow GEMM y = act(x B + b), B[k][n] = Bp[k sk + n sn]; K in {32, 36, 64, 100, 128}, 4 < N <= 112
bool narrowf_supported(int K, int N);
// fp32 y = act(x B + b) for K % 4 == 0, K <= 320, any N > 4 (B staged in LDS per 112-column block):
// the shapes narrowf cannot hold in registers (conv critic im2col GEMMs and their input gradients)
bool widef_supported(int K, int N);
void launch_widef(const float* x, const float* B, int sk, int sn, const float* b, float* y, int M, int K, int N,
                  int act, hipStream_t s);
void launch_narrowf(const float* x, const float* B, int sk, int sn, const float* b, float* y, int M, int K, int N,
                    int act, hipStream_t s);
void launch_skinny_fwd(int dt, const void* x, const float* W, const float* b, void* y, int M, int K, int N, int act,
                       hipStream_t s);
size_t skinny_wgrad_workspace_floats(int M, int K, int N);
void launch_skinny_wgrad(int dt, const void* x, const void* d, float* gW, float* gb, int M, int K, int N, float* ws,
                         hipStream_t s);
void launch_skinny_dgrad(int dt, const void* d, const float* W, void* dx, int M, int K, int N, hipStream_t s);
// linear Dense(1) head forward y = x W + b that also adds gW += sum_r ds_r x_r, gb += sum_r ds_r for the
// known per-row loss gradient ds_r = wa (r < split) / wb (the Wasserstein critic loss): one pass over x.
// ws: skinny_fwd_cs_workspace_floats(M, K) floats (every element written).
bool skinny_fwd_cs_supported(int K);
size_t skinny_fwd_cs_workspace_floats(int M, int K);
void launch_skinny_fwd_cs(int dt, const void* x, const float* W, const float* b, void* y, int M, int K, int split,
                          float wa, float wb, float* gW, float* gb, float* ws, hipStream_t s);
// a[0..na) += sum_z slab[z][0..na), b[0..nb) += sum_z slab[z][na..na+nb)  (fixed order; a/b may be null)
void launch_split_reduce(const float* slab, float* a, float* b, int splits, int na, int nb, hipStream_t s);

// ---- misc.hip ----
int device_cu_count();  // compute units of the current device (cached)
void launch_im2col_causal(int dt, const void* x, void* cols, int B, int Tn, int C, int k, int dil, hipStream_t s);
void launch_col2im_causal(int dt, const void* dcols, void* dx, int B, int Tn, int C, int k, int dil, hipStream_t s);
void launch_act_fwd(int dt, const void* x, void* y, int64_t n, int act, hipStream_t s);
void launch_act_bwd(int dt, const void* dy, const void* y, void* dx, int64_t n, int act, hipStream_t s);
void launch_act_tangent_bwd(int dt, const void* dyd, const void* y, const void* zd, void* out, int64_t n, int act,
                            hipStream_t s);
void launch_layernorm_fwd(int dt, const void* x, const float* gamma, const float* beta, void* y, void* xhat,
                          float* rstd, int64_t rows, int D, float eps, float pre_alpha, hipStream_t s);
// ggamma/gbeta (either may be null) += column sums via per-workgroup slabs in ws
// (layernorm_bwd_splits(rows) * 2 * D floats) and a fixed-order reduce: deterministic
int layernorm_bwd_splits(int64_t rows);
void launch_layernorm_bwd(int dt, const void* dy, const void* xhat, const float* rstd, const float* gamma,
                          void* dx, float* ggamma, float* gbeta, float* ws, int64_t rows, int D, hipStream_t s);
// LayerNorm JVP (yd = gamma * xhat') and its reverse (dy may be null = zero primal seed; dx / dxd
// both null = parameter gradients only); ggamma / gbeta accumulate through the same slab scheme
void launch_layernorm_tfwd(int dt, const void* xd, const void* xhat, const float* rstd, const float* gamma, void* yd,
                           int64_t rows, int D, hipStream_t s);
void launch_layernorm_tbwd(int dt, const void* dy, const void* dyd, const void* xd, const void* xhat,
                           const float* rstd, const float* gamma, void* dx, void* dxd, float* ggamma, float* gbeta,
                           float* ws, int64_t rows, int D, hipStream_t s);
// v = dGP/dg per row, pen += sum_b (1 - |g_b|)^2 / B  (rowpen: B floats of workspace)
void launch_gan_loss(int dt, const void* p, int64_t n, int64_t split, float la, float lb, int kind, void* grad,
                     float* partial, float* out, hipStream_t s);
int gan_loss_partials();
void launch_gp_pack(const float* pen, const float* w, float weight, float* pack, hipStream_t s);
void launch_gp_coef(int dt, const void* g, void* v, float* pen, float* rowpen, int B, int64_t D, float weight,
                    hipStream_t s, const float* w = nullptr, float* pack = nullptr);
void launch_interpolate(int dt, const void* real, const void* fake, const float* alpha, void* out, int B,
                        int64_t D, hipStream_t s);
void launch_philox_fill(int dt, void* out, int64_t n, uint64_t seed, int64_t* ctr, int dist, hipStream_t s);
void launch_sample_windows(int dt, const float* data, int64_t N, int64_t D, void* out, int B, uint64_t seed,
                           int64_t* ctr, hipStream_t s);
void launch_cast(int dt_in, const void* in, int dt_out, void* out, int64_t n, hipStream_t s);

// ---- optim.hip ----
void launch_rmsprop(float* p, const float* g, float* ms, int64_t n, float lr, float rho, float eps, float clip,
                    float gscale, hipStream_t s);
void launch_adam(float* p, const float* g, float* m, float* v, int64_t n, const float* step, float lr, float b1,
                 float b2, float eps, float clip, float gscale, hipStream_t s);
void launch_nadam(float* p, const float* g, float* m, float* v, int64_t n, const float* step, const float* m_cache,
                  float lr, float b1, float b2, float eps, float gscale, hipStream_t s);
void launch_step_advance(float* step, float* m_cache, float b1, hipStream_t s);
void launch_clip(float* p, int64_t n, float c, hipStream_t s);

// ---- p2p.hip: one-shot all-reduce over IPC-mapped peer buffers (layout in p2p.hip) ----
constexpr int kP2PMaxRanks = 8, kP2PMaxBlocks = 256;
constexpr int kP2PCtr = 0, kP2PDone = 128, kP2PErr = 256, kP2PFlags = 4096, kP2PData = 16384;
struct P2PPeers { char* base[kP2PMaxRanks]; };  // every rank's buffer as mapped in this process
size_t p2p_buffer_bytes(int64_t cap);
void* p2p_alloc(int64_t cap, int device, bool* fine_grained);  // zeroed; throws std::runtime_error
void p2p_free(void* p);
void p2p_ipc_handle(void* p, uint8_t out[64]);
void* p2p_ipc_open(const uint8_t h[64], int device);
void p2p_ipc_close(void* p);
int p2p_read_error(void* own);  // the sticky error word: 0, or 1 + the rank that gave up first (synchronous)
uint64_t p2p_timeout_ticks(double seconds, int device);  // seconds -> wall-clock (s_memrealtime) ticks
int p2p_blocks(int64_t n);
// x[0 .. n) = scale * sum over ranks (rank order) of every rank's x; n <= cap, same n on every rank
void launch_p2p_allreduce(float* x, int64_t n, const P2PPeers& peers, int rank, int world, int64_t cap, float scale,
                          uint64_t timeout_ticks, hipStream_t s);

}  // namespace hfrep
