// Offline schedule model (r03): batched pull rounds as the GPU runs them --
// a round visits the vertices in an order, W at a time (the concurrency window: a window
// reads the values at its start), a vertex is visited when an in-neighbour changed -- with
// the order reversed on alternate rounds (dir 2/3), same-round activation of later vertices
// (eager), and vertex orders by id / degree / random.  Counts rounds, visits per (vertex,
// batch) and 512-B tail-row reads per arc (KL lanes per batch: -DKL=16 etc.).
// usage: sched_sim_gs graph.bin W dir eager order [batches]   (graph.bin: export_csr.py)
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define KL 64
static int32_t V; static int64_t M; static int64_t* ptr; static int32_t* src; static double* w;
static int32_t nsrc; static int32_t* srcs;
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  fread(&V, 4, 1, f); fread(&M, 8, 1, f);
  ptr = malloc(8 * (V + 1)); src = malloc(4 * M); w = malloc(8 * M);
  fread(ptr, 8, V + 1, f); fread(src, 4, M, f); fread(w, 8, M, f);
  fread(&nsrc, 4, 1, f); srcs = malloc(4 * nsrc); fread(srcs, 4, nsrc, f); fclose(f);
  int W = atoi(argv[2]);          // window (vertices processed concurrently)
  int dirmode = atoi(argv[3]);    // 0 forward, 1 reverse, 2 alternate (fwd first), 3 alternate (rev first)
  int eager = atoi(argv[4]);      // same-round activation of later vertices
  int ordmode = atoi(argv[5]);    // 0 identity, 1 degree desc, 2 random
  int nbatch = argc > 6 ? atoi(argv[6]) : 4;
  int32_t* pos = malloc(4 * V); int32_t* ord = malloc(4 * V);
  for (int i = 0; i < V; i++) ord[i] = i;
  if (ordmode == 1) { // degree desc (stable)
    int64_t* k = malloc(8 * V);
    for (int i = 0; i < V; i++) k[i] = -(ptr[i + 1] - ptr[i]) * (int64_t)V * 4 + i;
    // simple sort via qsort on pairs
    int cmp(const void* a, const void* b) { int64_t x = k[*(int32_t*)a], y = k[*(int32_t*)b]; return x < y ? -1 : x > y; }
    qsort(ord, V, 4, cmp);
  } else if (ordmode == 2) {
    srand(1); for (int i = V - 1; i > 0; i--) { int j = rand() % (i + 1); int t = ord[i]; ord[i] = ord[j]; ord[j] = t; }
  }
  for (int i = 0; i < V; i++) pos[ord[i]] = i;
  double* D = malloc(8 * (size_t)V * KL); double* Dn = malloc(8 * (size_t)KL * W);
  uint8_t* act[2] = {calloc(V, 1), calloc(V, 1)};
  int32_t* chg = malloc(4 * W);
  double tot_rounds = 0, tot_visits = 0, tot_rows = 0;
  int nb_total = nsrc / KL;
  for (int bi = 0; bi < nbatch; bi++) {
    int b = (int)((long)bi * nb_total / nbatch);
    const int32_t* s = srcs + b * KL;
    for (size_t i = 0; i < (size_t)V * KL; i++) D[i] = INFINITY;
    memset(act[0], 0, V); memset(act[1], 0, V);
    for (int l = 0; l < KL; l++) { int v = s[l]; D[(size_t)v * KL + l] = 0; for (int64_t x = ptr[v]; x < ptr[v + 1]; x++) act[0][src[x]] = 1; }
    long rounds = 0, visits = 0, rows = 0;
    for (int r = 0;; r++) {
      uint8_t* ac = act[r & 1]; uint8_t* an = act[(r + 1) & 1];
      int any = 0; for (int i = 0; i < V; i++) if (ac[i]) { any = 1; break; }
      if (!any) break;
      rounds++;
      int rev = dirmode == 1 || (dirmode == 2 && (r & 1)) || (dirmode == 3 && !(r & 1));
      for (int c0 = 0; c0 < V; c0 += W) {
        int c1 = c0 + W < V ? c0 + W : V; int nc = 0;
        for (int p = c0; p < c1; p++) {
          int v = ord[rev ? V - 1 - p : p];
          if (!ac[v]) continue;
          ac[v] = 0; visits++; rows += ptr[v + 1] - ptr[v];
          double* out = Dn + (size_t)(p - c0) * KL; int changed = 0;
          for (int l = 0; l < KL; l++) {
            double bst = D[(size_t)v * KL + l];
            if (s[l] != v)
              for (int64_t x = ptr[v]; x < ptr[v + 1]; x++) { double c = D[(size_t)src[x] * KL + l] + w[x]; if (c < bst) bst = c; }
            out[l] = bst; if (bst != D[(size_t)v * KL + l]) changed = 1;
          }
          if (changed) chg[nc++] = p;
        }
        for (int i = 0; i < nc; i++) {
          int p = chg[i]; int v = ord[rev ? V - 1 - p : p];
          memcpy(D + (size_t)v * KL, Dn + (size_t)(p - c0) * KL, 8 * KL);
          for (int64_t x = ptr[v]; x < ptr[v + 1]; x++) { // undirected: out = in
            int u = src[x]; an[u] = 1;
            if (eager) { int pu = rev ? V - 1 - pos[u] : pos[u]; if (pu >= c1) ac[u] = 1; }
          }
        }
      }
    }
    tot_rounds += rounds; tot_visits += visits; tot_rows += rows;
  }
  printf("W=%d dir=%d eager=%d ord=%d: rounds %.1f visits/v %.2f rows/arc %.2f\n", W, dirmode, eager, ordmode,
         tot_rounds / nbatch, tot_visits / nbatch / V, tot_rows / nbatch / M);
  return 0;
}
