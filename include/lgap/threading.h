// Thread count of the library's OpenMP regions (reference include/LightGBM/utils/
// openmp_wrapper.h:11-47 and src/utils/openmp_wrapper.cpp): the `num_threads` parameter
// sets the default (<= 0: OpenMP's own default), LGBM_SetMaxThreads caps it. The
// effective count is pushed into OpenMP's default team size, which every parallel
// region of the library uses.
#pragma once

namespace lgap {

void SetDefaultNumThreads(int num_threads);
void SetMaxNumThreads(int num_threads);
int MaxNumThreadsSetting();  // LGBM_GetMaxThreads: the cap, -1 when none
int NumThreads();            // effective team size
void ApplyNumThreads();      // the effective team size -> the calling thread's OpenMP setting

}  // namespace lgap
