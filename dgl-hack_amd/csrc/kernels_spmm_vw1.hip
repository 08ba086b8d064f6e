// g-SpMM chunk kernels for rows of single-float slots (odd F, or a broadcast head
// width that is odd): see kernels_spmm.hip.
#include "spmm_chunk.h"

namespace dglmi {

void launch_fast_chunk_vw1(int kind, int red, const FastArgs& a, hipStream_t s) {
  const IdxPtr indptr = a.indptr;
  switch (kind) {
    case FAST_COPY_COL:
      if (red == RED_MAX) run_vw<FAST_COPY_COL, RED_MAX, 1>(a, indptr, s);
      else if (red == RED_MIN) run_vw<FAST_COPY_COL, RED_MIN, 1>(a, indptr, s);
      else run_vw<FAST_COPY_COL, RED_SUM, 1>(a, indptr, s);
      break;
    case FAST_COPY_EDGE:
      if (red == RED_MAX) run_vw<FAST_COPY_EDGE, RED_MAX, 1>(a, indptr, s);
      else if (red == RED_MIN) run_vw<FAST_COPY_EDGE, RED_MIN, 1>(a, indptr, s);
      else run_vw<FAST_COPY_EDGE, RED_SUM, 1>(a, indptr, s);
      break;
    case FAST_COL_MUL_EDGE: run_vw<FAST_COL_MUL_EDGE, RED_SUM, 1>(a, indptr, s); break;
    case FAST_COL_TIE: run_vw<FAST_COL_TIE, RED_SUM, 1>(a, indptr, s); break;
    default: run_vw<FAST_COL_MUL_EDGE_BCAST, RED_SUM, 1>(a, indptr, s); break;
  }
}

}  // namespace dglmi
