/*
 * cpu_ref.c — C99/OpenMP restatement of the reference CPU fusion path — TEST INFRASTRUCTURE ONLY.
 *
 * Used only by tests/ (cross-check against the numpy oracle) and by bench.py's cpu_baseline leg
 * (timed on the host cores). Never linked into the product.
 *
 * Per voxel, exactly the numpy/numba dtype flow of
 *   vox2world             fusion_with_occlusion/tsdf.py:338-349   (f32 origin + f64 vs*i -> f32)
 *   ED_warp               NonRigidICP/model/geometry.py:9-25      (f32, reference op order)
 *   cam2pix / visibility  tsdf.py:351-364, 576-612                (f64, round-half-even)
 *   integrate_tsdf        tsdf.py:366-376, 442-476                (f64 update, f32 store)
 *   colour average        tsdf.py:479-494                         (f32)
 * Build: gcc -O2 -fopenmp -ffp-contract=off -shared -fPIC (see oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <omp.h>

static inline float cdiv(float a, float b) { return (float)((double)a / (double)b); }

int64_t ofxref_integrate(int Dx, int Dy, int Dz, const float* origin, double vs,
                         const int64_t* vox, int64_t n_vox,              /* linear C-order voxel ids */
                         int warp, const int32_t* anchors, const float* weights, const uint8_t* valid, int K,
                         const float* R, const float* T, const float* G, /* node-relative transforms */
                         const float* depth, const float* color_im, int W, int H,
                         float fx, float fy, float cx, float cy, double trunc, double obs,
                         float* tsdf, float* weight, float* color) {
  int64_t n_upd = 0;
  const double fxd = fx, fyd = fy, cxd = cx, cyd = cy;
#pragma omp parallel for schedule(static) reduction(+ : n_upd)
  for (int64_t s = 0; s < n_vox; ++s) {
    int64_t v = vox[s];
    int64_t k = v % Dz, r = v / Dz;
    int64_t j = r % Dy, i = r / Dy;
    (void)Dx;
    float x = (float)((double)origin[0] + vs * (double)i);
    float y = (float)((double)origin[1] + vs * (double)j);
    float z = (float)((double)origin[2] + vs * (double)k);
    if (warp) {
      if (!valid[s]) continue;
      float ax = 0.f, ay = 0.f, az = 0.f;
      for (int q = 0; q < K; ++q) {
        int a = anchors[s * K + q];
        float w = weights[s * K + q];
        const float* Rn = R + 9 * (int64_t)a;
        const float* g = G + 3 * (int64_t)a;
        const float* t = T + 3 * (int64_t)a;
        float dx = x - g[0], dy = y - g[1], dz = z - g[2];
        float rx = Rn[0] * dx; rx = rx + Rn[1] * dy; rx = rx + Rn[2] * dz;
        float ry = Rn[3] * dx; ry = ry + Rn[4] * dy; ry = ry + Rn[5] * dz;
        float rz = Rn[6] * dx; rz = rz + Rn[7] * dy; rz = rz + Rn[8] * dz;
        float yx = ((rx + g[0]) + t[0]) * w, yy = ((ry + g[1]) + t[1]) * w, yz = ((rz + g[2]) + t[2]) * w;
        if (q == 0) { ax = yx; ay = yy; az = yz; }
        else { ax = ax + yx; ay = ay + yy; az = az + yz; }
      }
      x = ax; y = ay; z = az;
    }
    double X = x, Y = y, Z = z;
    double u = rint((X * fxd) / Z + cxd), vv = rint((Y * fyd) / Z + cyd);
    if (!(u >= 0.0 && u < (double)W && vv >= 0.0 && vv < (double)H && Z > 0.0)) continue;
    int64_t pix = (int64_t)vv * W + (int64_t)u;
    float d = depth[pix];
    double dd = (double)d - Z;
    if (!(d > 0.f && dd >= -trunc)) continue;
    double dist = fmin(1.0, dd / trunc);
    float w_old = weight[v], t_old = tsdf[v];
    float w_new = (float)((double)w_old + obs);
    float prod = w_old * t_old;
    weight[v] = w_new;
    tsdf[v] = (float)(((double)prod + obs * dist) / (double)w_new);
    if (color) {
      const float C = 65536.0f;
      float oc = color[v];
      float ob = floorf(oc / C), og = floorf((oc - ob * C) / 256.0f), orr = (oc - ob * C) - og * 256.0f;
      float nc = color_im[pix];
      float nb = floorf(nc / C), ng = floorf((nc - nb * C) / 256.0f), nr = (nc - nb * C) - ng * 256.0f;
      float ow = (float)obs;
      float b2 = fminf(255.0f, rintf(cdiv(w_old * ob + ow * nb, w_new)));
      float g2 = fminf(255.0f, rintf(cdiv(w_old * og + ow * ng, w_new)));
      float r2 = fminf(255.0f, rintf(cdiv(w_old * orr + ow * nr, w_new)));
      color[v] = (b2 * C + g2 * 256.0f) + r2;
    }
    n_upd += 1;
  }
  return n_upd;
}

/* thread count of the OpenMP loop above (bench.py cpu_baseline: the 1-thread leg) */
void ofxref_set_threads(int n) { omp_set_num_threads(n); }
