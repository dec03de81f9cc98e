/* Test harness (tests/test_pspt_host.py): the product's pspt dialogue and
 * file code (compton2d_amd/csrc/pspt_host.h, used by c2d_obs_begin_pspt /
 * c2d_obs_write_pspt) exported for a CPU check against compton2d_amd/
 * observer.py and the reference pspt's own output files. */
#include "../../compton2d_amd/csrc/pspt_host.h"

int pw_sizeof(void) { return (int)sizeof(c2d_pspt_deck); }
int pw_parse(const char* text, c2d_pspt_deck* d) { return c2d_pspt_parse(text, d); }
int pw_write(const char* path, const c2d_pspt_deck* d, const double* F, const double* cnt, int factor) {
  return c2d_pspt_write(path, d, F, cnt, factor);
}
