// Offline schedule model (r03): batched delta-stepping as threshold-gated pull
// rounds -- a lane's improvement at v propagates only once it is below the lane's bucket
// threshold T_s = off_s + k*delta (deferred otherwise), the bucket advancing when no
// propagation is left -- with per-lane offsets off_s = -d(s, max-degree hub) (mode 1) to
// align the 64 lanes' wavefronts.  Counts phases, rounds, visits and row reads per arc.
// usage: sched_sim_delta graph.bin delta offmode [batches] [sort-sources-by-offset]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define KL 64
#ifndef WIN
#define WIN 0  /* 0: Jacobi rounds; W > 0: a window of W vertices reads the values at its start */
#endif
static int32_t V; static int64_t M; static int64_t* ptr; static int32_t* src; static double* w;
static int32_t nsrc; static int32_t* srcs;
static void dijkstra1(int s, double* d) { // simple O(V^2)-free binary heap dijkstra
  int32_t* h = malloc(4 * V); int32_t* hp = malloc(4 * V); int n = 0;
  for (int i = 0; i < V; i++) { d[i] = INFINITY; hp[i] = -1; }
  d[s] = 0; h[n] = s; hp[s] = n++;
  #define SW(a,b) { int32_t t=h[a]; h[a]=h[b]; h[b]=t; hp[h[a]]=a; hp[h[b]]=b; }
  while (n) {
    int u = h[0]; n--; if (n) { h[0] = h[n]; hp[h[0]] = 0; int i = 0; for (;;) { int l = 2*i+1, r = l+1, m = i; if (l<n && d[h[l]]<d[h[m]]) m=l; if (r<n && d[h[r]]<d[h[m]]) m=r; if (m==i) break; SW(i,m); i=m; } }
    hp[u] = -2;
    for (int64_t x = ptr[u]; x < ptr[u+1]; x++) { int v = src[x]; double c = d[u] + w[x];
      if (c < d[v]) { d[v] = c; if (hp[v] == -1) { h[n] = v; hp[v] = n++; } int i = hp[v]; while (i && d[h[(i-1)/2]] > d[h[i]]) { SW(i,(i-1)/2); i=(i-1)/2; } } }
  }
  free(h); free(hp);
}
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  if (fread(&V, 4, 1, f) != 1 || fread(&M, 8, 1, f) != 1) return 1;
  ptr = malloc(8 * (V + 1)); src = malloc(4 * M); w = malloc(8 * M);
  if (fread(ptr, 8, V + 1, f) != (size_t)V + 1 || fread(src, 4, M, f) != (size_t)M || fread(w, 8, M, f) != (size_t)M) return 1;
  if (fread(&nsrc, 4, 1, f) != 1) return 1; srcs = malloc(4 * nsrc); if (fread(srcs, 4, nsrc, f) != (size_t)nsrc) return 1; fclose(f);
  double delta = atof(argv[2]);
  int offmode = atoi(argv[3]);   // 0 none, 1 d(s, max-degree vertex), 2 d(s, nearest of top-8 hubs)?
  int nbatch = argc > 4 ? atoi(argv[4]) : 4;
  int sortsrc = argc > 5 ? atoi(argv[5]) : 0;  // sort attached by offset before batching
  int hub = 0; for (int i = 1; i < V; i++) if (ptr[i+1]-ptr[i] > ptr[hub+1]-ptr[hub]) hub = i;
  double* dh = malloc(8 * V); dijkstra1(hub, dh);
  int32_t* S = malloc(4 * nsrc); memcpy(S, srcs, 4 * nsrc);
  if (sortsrc) { int cmp(const void* a, const void* b) { double x = dh[*(int32_t*)a], y = dh[*(int32_t*)b]; return x < y ? -1 : x > y; } qsort(S, nsrc, 4, cmp); }
  double* D = malloc(8 * (size_t)V * KL); double* Dn = malloc(8 * (size_t)V * KL);
  uint8_t* act = calloc(V, 1); uint8_t* actn = calloc(V, 1); uint64_t* pend = calloc(V, 8);
  double tr = 0, tv = 0, trow = 0, tph = 0;
  int nbt = nsrc / KL;
  for (int bi = 0; bi < nbatch; bi++) {
    int b = (int)((long)bi * nbt / nbatch); const int32_t* s = S + b * KL;
    double T[KL], off[KL];
    for (int l = 0; l < KL; l++) { off[l] = offmode ? -dh[s[l]] : 0; T[l] = off[l] + delta; }
    for (size_t i = 0; i < (size_t)V * KL; i++) D[i] = INFINITY;
    memset(act, 0, V); memset(pend, 0, 8 * V);
    for (int l = 0; l < KL; l++) { D[(size_t)s[l] * KL + l] = 0; pend[s[l]] |= 1ull << l; }
    long rounds = 0, visits = 0, rows = 0, phases = 0;
    for (;;) {
      // release pending lanes under threshold
      int anyp = 0, anya = 0;
      for (int v = 0; v < V; v++) if (pend[v]) {
        anyp = 1; uint64_t rel = 0;
        for (int l = 0; l < KL; l++) if ((pend[v] >> l & 1) && D[(size_t)v*KL+l] < T[l]) rel |= 1ull << l;
        if (rel) { pend[v] &= ~rel; for (int64_t x = ptr[v]; x < ptr[v+1]; x++) { act[src[x]] = 1; anya = 1; } }
      }
      if (!anyp && !anya) break;
      if (!anya) { for (int l = 0; l < KL; l++) T[l] += delta; phases++; continue; }
      phases++;
      while (anya) {  // rounds within the phase (Jacobi, or Gauss-Seidel with window W)
        rounds++; anya = 0; memset(actn, 0, V);
        memcpy(Dn, D, 8 * (size_t)V * KL);
        for (int v = 0; v < V; v++) {
          if (WIN > 0 && v % WIN == 0 && v) memcpy(D + (size_t)(v - WIN) * KL, Dn + (size_t)(v - WIN) * KL, 8 * (size_t)WIN * KL);
          if (!act[v]) continue;
          act[v] = 0; visits++; rows += ptr[v+1]-ptr[v];
          uint64_t prop = 0;
          for (int l = 0; l < KL; l++) { if (s[l] == v) continue; double bst = D[(size_t)v*KL+l];
            for (int64_t x = ptr[v]; x < ptr[v+1]; x++) { double c = D[(size_t)src[x]*KL+l] + w[x]; if (c < bst) bst = c; }
            if (bst != D[(size_t)v*KL+l]) { Dn[(size_t)v*KL+l] = bst; if (bst < T[l]) { prop |= 1ull << l; pend[v] &= ~(1ull << l); } else pend[v] |= 1ull << l; } }
          if (prop) for (int64_t x = ptr[v]; x < ptr[v+1]; x++) actn[src[x]] = 1;
        }
        memcpy(D, Dn, 8 * (size_t)V * KL);
        for (int v = 0; v < V; v++) if (actn[v]) { act[v] = 1; anya = 1; }
      }
      for (int l = 0; l < KL; l++) T[l] += delta;
    }
    tr += rounds; tv += visits; trow += rows; tph += phases;
  }
  printf("delta=%g off=%d sort=%d: phases %.1f rounds %.1f visits/v %.2f rows/arc %.2f\n", delta, offmode, sortsrc,
         tph / nbatch, tr / nbatch, tv / nbatch / V, trow / nbatch / M);
  return 0;
}
