// CORE_redistribute_dtd (include/parsec/data_dist/matrix/redistribute/
// redistribute_internal.h): the per-tile copy of a sub-matrix share that the
// reference's redistribute test JDFs call (tests/collections/redistribute/
// redistribute_check.jdf:96,160; reference redistribute_dtd.c:49-110). One
// rule instead of the nine corner / bar / inner cases: a tile's rows start at
// i_start in the first tile row of the sub-matrix and at 0 elsewhere, and end
// at i_end in the last one (at mb_T_inner rows when it is also the first);
// columns the same way.
#include <algorithm>
#include <cstring>

extern "C" void CORE_redistribute_dtd(double* T, double* Y, int mb_Y, int nb_Y, int m_Y, int n_Y, int m_Y_start, int m_Y_end, int n_Y_start, int n_Y_end,
                                      int i_start, int i_end, int j_start, int j_end, int mb_T, int mb_T_inner, int nb_T_inner, int R, int i_start_T,
                                      int j_start_T) {
  const int rows_in = mb_Y - 2 * R, cols_in = nb_Y - 2 * R;
  auto span = [](int idx, int first, int last, int start, int end, int inner, int bound, int* off, int* count) {
    if (idx < first || idx > last) return false;
    *off = idx == first ? start : 0;
    if (idx == first) *count = std::min(inner - start, bound);
    else if (idx == last) *count = end + 1;
    else *count = inner;
    return *count > 0;
  };
  int r0, nr, c0, nc;
  if (!span(m_Y, m_Y_start, m_Y_end, i_start, i_end, rows_in, mb_T_inner, &r0, &nr)) return;
  if (!span(n_Y, n_Y_start, n_Y_end, j_start, j_end, cols_in, nb_T_inner, &c0, &nc)) return;
  // position of the tile's share inside T: the rows / columns of the tiles before it
  const int ti = i_start_T + (m_Y == m_Y_start ? 0 : (m_Y - m_Y_start) * rows_in - i_start);
  const int tj = j_start_T + (n_Y == n_Y_start ? 0 : (n_Y - n_Y_start) * cols_in - j_start);
  for (int c = 0; c < nc; ++c)
    std::memcpy(T + (size_t)(tj + c) * mb_T + ti, Y + (size_t)(R + c0 + c) * mb_Y + R + r0, (size_t)nr * sizeof(double));
}
