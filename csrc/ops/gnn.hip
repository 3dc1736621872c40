// GATv2 embedder entry points (reference models.py:10-53 on PyG GATv2Conv, aggr='mean'): dispatch to
// the fused per-graph MFMA kernels and the column-sum reduction of their per-workgroup gradients.
//
//   <= 32 nodes    gnn_mf.hip  one wave per graph (Abilene, BtEurope: the headline configs)
//   33..64 nodes   gnn_mt.hip  one graph per workgroup, one wave per 32-node tile (50-node configs)
//   65..256 nodes  gnn_lg.hip  one graph per 512-thread workgroup, all convs in LDS, recomputing backward
//                              (200-node configs; H < 24 at 200 nodes, LDS-bound)
//
// All need F_in <= 16, an encoder + ONE shared process block (GSC's num_layers = 2) and unique
// (source, target) messages (mf / mt: H <= 32; lg: H <= 31 and the LDS budget).  Every other shape --
// wider embedders, other layer counts -- runs the layer-wise kernels (gsc_amd/ops/gnn_lw.py: MFMA GEMM
// node linears + per-node attention kernels); gsc_amd/ops/gnn.py routes by gnn_fused_fits.
//
// The backward writes one partial gradient row per workgroup (each element owned by one lane or
// summed over the workgroup's waves in a fixed order: no atomics, bitwise reproducible); a column
// sum reduces the rows.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gnn_args.h"

namespace py = pybind11;

namespace gsc {

bool gnn_mf_supported(int Fin, int H, int NM, int L, int n_blocks, const int* layer_of);
void gnn_mf_forward(const void* args, uintptr_t stream, int cus);
int gnn_mf_backward(const void* args, uintptr_t stream, int cus, int max_rows);
int gnn_mf_saved_bytes(const void* args);
bool gnn_mt_supported(int Fin, int H, int NM, int M, int L, int n_blocks, const int* layer_of);
void gnn_mt_forward(const void* args, uintptr_t stream, int cus);
int gnn_mt_backward(const void* args, uintptr_t stream, int cus, int max_rows);
int gnn_mt_saved_bytes(const void* args);
bool gnn_lg_supported(int Fin, int H, int NM, int P, int M, int L, int n_blocks, const int* layer_of);
void gnn_lg_forward(const void* args, uintptr_t stream, int cus);
int gnn_lg_backward(const void* args, uintptr_t stream, int cus, int max_rows);
std::vector<unsigned long long> gnn_lg_prof();

__global__ __launch_bounds__(256) void column_sum_kernel(const float* __restrict__ partials, float* __restrict__ out,
                                                         int rows, int cols) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (c < cols)
    for (int r = rg; r < rows; r += 8) s += partials[(long)r * cols + c];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < cols) {
    float t = 0.f;
    for (int k = 0; k < 8; ++k) t += red[k][cl];
    out[c] = t;
  }
}

static int n_blocks_of(const std::vector<int>& layer_of) {
  int maxb = 0;
  for (int b : layer_of) maxb = b > maxb ? b : maxb;
  return maxb + 1;
}

enum GnnPath { kPathNone = 0, kPathMf = 1, kPathMt = 2, kPathLg = 3 };

// GSC_GNN_LG=0: large graphs on the layer-wise kernels instead (A/B)
static bool lg_enabled() {
  const char* e = getenv("GSC_GNN_LG");
  return !(e && e[0] == '0');
}

static GnnPath fused_path(int M, int NM, int P, int Fin, int H, const std::vector<int>& layer_of, bool uniq) {
  if (!uniq || layer_of.empty() || (int)layer_of.size() > kClMaxLayers) return kPathNone;
  const int L = (int)layer_of.size(), nb = n_blocks_of(layer_of);
  if (gnn_mf_supported(Fin, H, NM, L, nb, layer_of.data())) return kPathMf;
  // 33 .. 64-node graphs: packs of the large-graph kernels (several graphs per workgroup, every conv in LDS)
  if (NM > 32 && lg_enabled() && gnn_lg_supported(Fin, H, NM, P, M, L, nb, layer_of.data())) return kPathLg;
  if (gnn_mt_supported(Fin, H, NM, M, L, nb, layer_of.data())) return kPathMt;
  if (lg_enabled() && gnn_lg_supported(Fin, H, NM, P, M, L, nb, layer_of.data())) return kPathLg;
  return kPathNone;
}

static ClArgs make_args(py::dict t, uintptr_t params, uintptr_t x, uintptr_t topo, int B, int P, int Fin, int H,
                        const std::vector<int>& layer_of, GnnPath* path) {
  GSC_CHECK(!layer_of.empty() && (int)layer_of.size() <= kClMaxLayers, "1..16 conv applications");
  ClArgs c{};
  c.params = ptr<const float>(params);
  c.x = ptr<const float>(x);
  c.topo = ptr<const int32_t>(topo);
  c.in_src = ptr<const int32_t>(t["in_src"].cast<uintptr_t>());
  c.in_dst = ptr<const int32_t>(t["in_dst"].cast<uintptr_t>());
  c.in_ptr = ptr<const int32_t>(t["in_ptr"].cast<uintptr_t>());
  c.out_q = ptr<const int32_t>(t["out_q"].cast<uintptr_t>());
  c.out_ptr = ptr<const int32_t>(t["out_ptr"].cast<uintptr_t>());
  c.out_dst = ptr<const int32_t>(t["out_dst"].cast<uintptr_t>());
  c.deg = ptr<const float>(t["deg"].cast<uintptr_t>());
  c.nnodes = ptr<const int32_t>(t["nnodes"].cast<uintptr_t>());
  c.nmsgs = ptr<const int32_t>(t["nmsgs"].cast<uintptr_t>());
  c.s_dst = reinterpret_cast<const void*>(t["s_dst"].cast<uintptr_t>());
  c.s_src = reinterpret_cast<const void*>(t["s_src"].cast<uintptr_t>());
  c.MP = t["MP"].cast<int>();
  c.deg_order = t.contains("deg_order") ? ptr<const int32_t>(t["deg_order"].cast<uintptr_t>()) : nullptr;
  c.M = t["M"].cast<int>();
  c.NM = t["NM"].cast<int>();
  c.B = B;
  c.P = P;
  c.Fin = Fin;
  c.H = H;
  c.L = (int)layer_of.size();
  for (int i = 0; i < c.L; ++i) c.layer_of[i] = layer_of[i];
  c.n_blocks = n_blocks_of(layer_of);
  c.n_params = cl_block_offset(c.n_blocks - 1, Fin, H) + cl_block_size(c.n_blocks == 1 ? Fin : H, H);
  c.waves = 4;
  *path = fused_path(c.M, c.NM, P, Fin, H, layer_of, t["uniq"].cast<bool>());
  GSC_CHECK(*path != kPathNone,
            "GNN shape not covered by the fused MFMA kernels (route it to the layer-wise kernels, gnn_lw.py)");
  return c;
}

// CUs the launching stream may use: the device's count, or the budget of a CU-masked learner
// stream (gnn_set_cu_budget) so persistent grids are sized to one full round on that partition.
static int g_cu_budget = 0;
// Work-queue counters of the multi-tile backward (one zeroed slot per launch, rotating; allocated with the
// budget -- before any HIP-graph capture -- so a captured launch keeps its own slot and memset node)
static int* g_work = nullptr;
constexpr int kWorkSlots = 4096, kWorkCaptured = 3072;
static int g_work_cap = 0;        // slots [0, kWorkCaptured): one per launch recorded into a HIP graph, never reused
static unsigned g_work_eager = 0;  // slots [kWorkCaptured, kWorkSlots): eager launches, rotating (stream-ordered)
// A zeroed counter slot for one launch on `st` (the memset is enqueued / captured with it), or null
// (fixed-stride grid).  Captured launches get slots of their own: an eager launch on another stream
// (the act path) must never share a counter with a replayed one.
static int* work_slot(hipStream_t st) {
  if (!g_work || g_cu_budget <= 0) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  GSC_HIP_CHECK(hipStreamIsCapturing(st, &cs));
  int slot;
  if (cs == hipStreamCaptureStatusActive) {
    if (g_work_cap >= kWorkCaptured) {
      // (slots of destroyed graphs are not recycled: a long run of re-captures ends up here)
      static bool warned = false;
      if (!warned) {
        warned = true;
        fprintf(stderr, "[gsc_amd] gnn: %d captured work-queue slots used up; further captured launches use "
                        "the fixed-stride grid (slower)\n", kWorkCaptured);
      }
      return nullptr;
    }
    slot = g_work_cap++;
  } else {
    slot = kWorkCaptured + (int)(g_work_eager++ % (kWorkSlots - kWorkCaptured));
  }
  int* p = g_work + slot;
  GSC_HIP_CHECK(hipMemsetAsync(p, 0, sizeof(int), st));
  return p;
}
static int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    GSC_HIP_CHECK(hipGetDevice(&dev));
    GSC_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return cus;
}
void gnn_set_cu_budget(int n) {
  g_cu_budget = n > 0 ? n : 0;
  const char* e = getenv("GSC_GNN_WORKQ");
  if (g_cu_budget > 0 && !g_work && !(e && e[0] == '0'))
    GSC_HIP_CHECK(hipMalloc(&g_work, sizeof(int) * kWorkSlots));
}
static int num_cus() {
  const int cus = device_cus();
  return g_cu_budget > 0 && g_cu_budget < cus ? g_cu_budget : cus;
}

// Multi-tile forward: full-device grid claiming graphs from a fresh counter slot when a CU budget is set
// (overlap mode, see gnn_backward), else the fixed-stride grid
static void mt_forward_queued(ClArgs c, uintptr_t stream) {
  c.work = work_slot(stream_of(stream));
  if (c.work) {
    gnn_mt_forward(&c, stream, device_cus());
  } else {
    gnn_mt_forward(&c, stream, num_cus());
  }
}

// Large-graph forward: the same overlap-mode work queue (full-device grid claiming graphs)
static void lg_forward_queued(ClArgs c, uintptr_t stream) {
  c.work = work_slot(stream_of(stream));
  gnn_lg_forward(&c, stream, c.work ? device_cus() : num_cus());
}

void gnn_forward(py::dict tables, uintptr_t params, uintptr_t x, uintptr_t topo, uintptr_t emb, int B, int P, int Fin,
                 int H, std::vector<int> layer_of, uintptr_t stream, uintptr_t blob) {
  GnnPath path;
  ClArgs c = make_args(tables, params, x, topo, B, P, Fin, H, layer_of, &path);
  c.emb = ptr<float>(emb);
  c.blob = reinterpret_cast<void*>(blob);
  if (path == kPathMf) gnn_mf_forward(&c, stream, num_cus());
  else if (path == kPathLg) lg_forward_queued(c, stream);
  else mt_forward_queued(c, stream);
}

// Two parameter sets on the same graphs (target actor + target critic embedders of next_obs).  One-tile
// graphs: one launch of 8-wave workgroups holding both weight sets (headline: 108.0k vs 107.2k
// env-steps/s with two launches).  Two-tile graphs: two launches -- the second weight set's LDS costs
// the multi-tile kernel a resident workgroup per CU (syn50: 10.1k fused vs 10.6k env-steps/s).
void gnn_forward2(py::dict tables, uintptr_t params, uintptr_t params2, uintptr_t x, uintptr_t topo, uintptr_t emb,
                  uintptr_t emb2, int B, int P, int Fin, int H, std::vector<int> layer_of, uintptr_t stream) {
  GnnPath path;
  ClArgs c = make_args(tables, params, x, topo, B, P, Fin, H, layer_of, &path);
  c.emb = ptr<float>(emb);
  if (path == kPathMf) {
    c.params2 = ptr<const float>(params2);
    c.emb2 = ptr<float>(emb2);
    gnn_mf_forward(&c, stream, num_cus());
    return;
  }
  if (path == kPathLg) {
    lg_forward_queued(c, stream);
    c.params = ptr<const float>(params2);
    c.emb = ptr<float>(emb2);
    lg_forward_queued(c, stream);
    return;
  }
  mt_forward_queued(c, stream);
  c.params = ptr<const float>(params2);
  c.emb = ptr<float>(emb2);
  mt_forward_queued(c, stream);
}

void gnn_backward(py::dict tables, uintptr_t params, uintptr_t x, uintptr_t topo, uintptr_t demb, uintptr_t partials,
                  int max_rows, uintptr_t grad_out, int B, int P, int Fin, int H, std::vector<int> layer_of,
                  uintptr_t stream, uintptr_t blob) {
  GnnPath path;
  ClArgs c = make_args(tables, params, x, topo, B, P, Fin, H, layer_of, &path);
  c.demb = ptr<const float>(demb);
  c.partials = ptr<float>(partials);
  c.blob = reinterpret_cast<void*>(blob);
  int rows;
  if (path == kPathMf) {
    rows = gnn_mf_backward(&c, stream, num_cus(), max_rows);
  } else if (path == kPathLg) {  // recomputes the forward: no saved state; work queue in overlap mode
    c.work = work_slot(stream_of(stream));
    rows = gnn_lg_backward(&c, stream, c.work ? device_cus() : num_cus(), max_rows);
  } else if ((c.work = work_slot(stream_of(stream))) != nullptr) {
    // CU-masked partner stream (overlap mode): the grid spans every CU and claims graphs from a counter,
    // so the CUs the simulator releases mid-kernel join in (a fixed-stride grid sized to the budget left
    // them idle until the next launch)
    rows = gnn_mt_backward(&c, stream, device_cus(), max_rows);
  } else {
    rows = gnn_mt_backward(&c, stream, num_cus(), max_rows);
  }
  hipLaunchKernelGGL(column_sum_kernel, dim3((c.n_params + 31) / 32), dim3(256), 0, stream_of(stream),
                     (const float*)c.partials, ptr<float>(grad_out), rows, c.n_params);
  check_launch();
}

// Whether the fused MFMA kernels cover this shape (else: layer-wise kernels).
bool gnn_fused_fits(int M, int NM, int P, int Fin, int H, std::vector<int> layer_of, bool uniq) {
  return P >= NM && fused_path(M, NM, P, Fin, H, layer_of, uniq) != kPathNone;
}

// Bytes per graph the grad-requiring forward saves for the backward.
int gnn_saved_bytes(py::dict tables, int P, int Fin, int H, std::vector<int> layer_of) {
  GnnPath path;
  const ClArgs c = make_args(tables, 0, 0, 0, 1, P, Fin, H, layer_of, &path);
  if (path == kPathLg) return 0;
  return path == kPathMf ? gnn_mf_saved_bytes(&c) : gnn_mt_saved_bytes(&c);
}

int gnn_num_params(int Fin, int H, int max_block) {
  return cl_block_offset(max_block, Fin, H) + cl_block_size(max_block == 0 ? Fin : H, H);
}

void register_gnn(py::module_& m) {
  m.def("gnn_forward", &gnn_forward, py::arg("tables"), py::arg("params"), py::arg("x"), py::arg("topo"), py::arg("emb"),
        py::arg("B"), py::arg("P"), py::arg("Fin"), py::arg("H"), py::arg("layer_of"), py::arg("stream"),
        py::arg("blob") = 0);
  m.def("gnn_forward2", &gnn_forward2, py::arg("tables"), py::arg("params"), py::arg("params2"), py::arg("x"),
        py::arg("topo"), py::arg("emb"), py::arg("emb2"), py::arg("B"), py::arg("P"), py::arg("Fin"), py::arg("H"),
        py::arg("layer_of"), py::arg("stream"));
  m.def("gnn_backward", &gnn_backward, py::arg("tables"), py::arg("params"), py::arg("x"), py::arg("topo"),
        py::arg("demb"), py::arg("partials"), py::arg("max_rows"), py::arg("grad_out"), py::arg("B"), py::arg("P"),
        py::arg("Fin"), py::arg("H"), py::arg("layer_of"), py::arg("stream"), py::arg("blob") = 0);
  m.def("gnn_saved_bytes", &gnn_saved_bytes, "per-graph bytes of the forward state saved for the MFMA backward");
  m.def("gnn_num_params", &gnn_num_params);
  m.def("gnn_fused_fits", &gnn_fused_fits, py::arg("M"), py::arg("NM"), py::arg("P"), py::arg("Fin"), py::arg("H"),
        py::arg("layer_of"), py::arg("uniq"));
  m.def("gnn_set_cu_budget", &gnn_set_cu_budget, "CUs available to GNN launches (0 = whole device)");
  m.def("gnn_lg_prof", &gnn_lg_prof, "large-graph kernels' phase cycles (GSC_LG_PROF=1), read and cleared");
}

}  // namespace gsc
