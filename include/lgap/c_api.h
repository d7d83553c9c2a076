/* LGBM_* compatible C ABI of LambdaGap-MI355X (reference: include/LightGBM/c_api.h).
 * Every function returns 0 on success and -1 on failure; LGBM_GetLastError()
 * returns the message. Handles are opaque pointers. */
#ifndef LGAP_C_API_H_
#define LGAP_C_API_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
#define LGAP_EXTERN_C extern "C"
#else
#define LGAP_EXTERN_C
#endif
#define LIGHTGBM_C_EXPORT LGAP_EXTERN_C __attribute__((visibility("default")))

typedef void* DatasetHandle;
typedef void* BoosterHandle;
typedef void* FastConfigHandle;

#define C_API_DTYPE_FLOAT32 (0)
#define C_API_DTYPE_FLOAT64 (1)
#define C_API_DTYPE_INT32 (2)
#define C_API_DTYPE_INT64 (3)

#define C_API_PREDICT_NORMAL (0)
#define C_API_PREDICT_RAW_SCORE (1)
#define C_API_PREDICT_LEAF_INDEX (2)
#define C_API_PREDICT_CONTRIB (3)

#define C_API_FEATURE_IMPORTANCE_SPLIT (0)
#define C_API_FEATURE_IMPORTANCE_GAIN (1)

LIGHTGBM_C_EXPORT const char* LGBM_GetLastError();
LIGHTGBM_C_EXPORT int LGBM_RegisterLogCallback(void (*callback)(const char*));
LIGHTGBM_C_EXPORT int LGBM_DumpParamAliases(int64_t buffer_len, int64_t* out_len, char* out_str);
LIGHTGBM_C_EXPORT int LGBM_GetSampleCount(int32_t num_total_row, const char* parameters, int* out);
LIGHTGBM_C_EXPORT int LGBM_SampleIndices(int32_t num_total_row, const char* parameters, void* out, int32_t* out_len);

/* ---- Dataset */
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromFile(const char* filename, const char* parameters,
                                                 const DatasetHandle reference, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromMat(const void* data, int data_type, int32_t nrow, int32_t ncol,
                                                int is_row_major, const char* parameters,
                                                const DatasetHandle reference, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromMats(int32_t nmat, const void** data, int data_type, int32_t* nrow,
                                                 int32_t ncol, int is_row_major, const char* parameters,
                                                 const DatasetHandle reference, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromCSR(const void* indptr, int indptr_type, const int32_t* indices,
                                                const void* data, int data_type, int64_t nindptr, int64_t nelem,
                                                int64_t num_col, const char* parameters,
                                                const DatasetHandle reference, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromCSC(const void* col_ptr, int col_ptr_type, const int32_t* indices,
                                                const void* data, int data_type, int64_t ncol_ptr, int64_t nelem,
                                                int64_t num_row, const char* parameters,
                                                const DatasetHandle reference, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateByReference(const DatasetHandle reference, int64_t num_total_row,
                                                    DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetInitStreaming(DatasetHandle dataset, int32_t has_weights, int32_t has_init_scores,
                                                int32_t has_queries, int32_t nclasses, int32_t nthreads,
                                                int32_t omp_max_threads);
LIGHTGBM_C_EXPORT int LGBM_DatasetPushRows(DatasetHandle dataset, const void* data, int data_type, int32_t nrow,
                                           int32_t ncol, int32_t start_row);
LIGHTGBM_C_EXPORT int LGBM_DatasetPushRowsWithMetadata(DatasetHandle dataset, const void* data, int data_type,
                                                       int32_t nrow, int32_t ncol, int32_t start_row,
                                                       const float* label, const float* weight,
                                                       const double* init_score, const int32_t* query, int32_t tid);
LIGHTGBM_C_EXPORT int LGBM_DatasetPushRowsByCSR(DatasetHandle dataset, const void* indptr, int indptr_type,
                                                const int32_t* indices, const void* data, int data_type,
                                                int64_t nindptr, int64_t nelem, int64_t num_col, int64_t start_row);
LIGHTGBM_C_EXPORT int LGBM_DatasetSetWaitForManualFinish(DatasetHandle dataset, int wait);
LIGHTGBM_C_EXPORT int LGBM_DatasetMarkFinished(DatasetHandle dataset);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetSubset(const DatasetHandle handle, const int32_t* used_row_indices,
                                            int32_t num_used_row_indices, const char* parameters, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetSetFeatureNames(DatasetHandle handle, const char** feature_names,
                                                  int num_feature_names);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetFeatureNames(DatasetHandle handle, const int len, int* num_feature_names,
                                                  const size_t buffer_len, size_t* out_buffer_len,
                                                  char** feature_names);
LIGHTGBM_C_EXPORT int LGBM_DatasetFree(DatasetHandle handle);
LIGHTGBM_C_EXPORT int LGBM_DatasetSaveBinary(DatasetHandle handle, const char* filename);
LIGHTGBM_C_EXPORT int LGBM_DatasetDumpText(DatasetHandle handle, const char* filename);
LIGHTGBM_C_EXPORT int LGBM_DatasetSetField(DatasetHandle handle, const char* field_name, const void* field_data,
                                           int num_element, int type);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetField(DatasetHandle handle, const char* field_name, int* out_len,
                                           const void** out_ptr, int* out_type);
LIGHTGBM_C_EXPORT int LGBM_DatasetUpdateParamChecking(const char* old_parameters, const char* new_parameters);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetNumData(DatasetHandle handle, int* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetNumFeature(DatasetHandle handle, int* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetGetFeatureNumBin(DatasetHandle handle, int feature, int* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetAddFeaturesFrom(DatasetHandle target, DatasetHandle source);

/* ---- Booster */
LIGHTGBM_C_EXPORT int LGBM_BoosterCreate(const DatasetHandle train_data, const char* parameters, BoosterHandle* out);
LIGHTGBM_C_EXPORT int LGBM_BoosterCreateFromModelfile(const char* filename, int* out_num_iterations,
                                                      BoosterHandle* out);
LIGHTGBM_C_EXPORT int LGBM_BoosterLoadModelFromString(const char* model_str, int* out_num_iterations,
                                                      BoosterHandle* out);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetLoadedParam(BoosterHandle handle, int64_t buffer_len, int64_t* out_len,
                                                 char* out_str);
LIGHTGBM_C_EXPORT int LGBM_BoosterFree(BoosterHandle handle);
LIGHTGBM_C_EXPORT int LGBM_BoosterShuffleModels(BoosterHandle handle, int start_iter, int end_iter);
LIGHTGBM_C_EXPORT int LGBM_BoosterMerge(BoosterHandle handle, BoosterHandle other_handle);
LIGHTGBM_C_EXPORT int LGBM_BoosterAddValidData(BoosterHandle handle, const DatasetHandle valid_data);
LIGHTGBM_C_EXPORT int LGBM_BoosterResetTrainingData(BoosterHandle handle, const DatasetHandle train_data);
LIGHTGBM_C_EXPORT int LGBM_BoosterResetParameter(BoosterHandle handle, const char* parameters);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetNumClasses(BoosterHandle handle, int* out_len);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetLinear(BoosterHandle handle, int* out);
LIGHTGBM_C_EXPORT int LGBM_BoosterUpdateOneIter(BoosterHandle handle, int* is_finished);
LIGHTGBM_C_EXPORT int LGBM_BoosterRefit(BoosterHandle handle, const int32_t* leaf_preds, int32_t nrow, int32_t ncol);
LIGHTGBM_C_EXPORT int LGBM_BoosterUpdateOneIterCustom(BoosterHandle handle, const float* grad, const float* hess,
                                                      int* is_finished);
LIGHTGBM_C_EXPORT int LGBM_BoosterRollbackOneIter(BoosterHandle handle);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetCurrentIteration(BoosterHandle handle, int* out_iteration);
LIGHTGBM_C_EXPORT int LGBM_BoosterNumModelPerIteration(BoosterHandle handle, int* out_tree_per_iteration);
LIGHTGBM_C_EXPORT int LGBM_BoosterNumberOfTotalModel(BoosterHandle handle, int* out_models);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetEvalCounts(BoosterHandle handle, int* out_len);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetEvalNames(BoosterHandle handle, const int len, int* out_len,
                                               const size_t buffer_len, size_t* out_buffer_len, char** out_strs);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetFeatureNames(BoosterHandle handle, const int len, int* out_len,
                                                  const size_t buffer_len, size_t* out_buffer_len, char** out_strs);
LIGHTGBM_C_EXPORT int LGBM_BoosterValidateFeatureNames(BoosterHandle handle, const char** data_names,
                                                       int data_num_features);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetNumFeature(BoosterHandle handle, int* out_len);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetEval(BoosterHandle handle, int data_idx, int* out_len, double* out_results);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetNumPredict(BoosterHandle handle, int data_idx, int64_t* out_len);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetPredict(BoosterHandle handle, int data_idx, int64_t* out_len, double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForFile(BoosterHandle handle, const char* data_filename,
                                                 int data_has_header, int predict_type, int start_iteration,
                                                 int num_iteration, const char* parameter,
                                                 const char* result_filename);
LIGHTGBM_C_EXPORT int LGBM_BoosterCalcNumPredict(BoosterHandle handle, int num_row, int predict_type,
                                                 int start_iteration, int num_iteration, int64_t* out_len);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForCSR(BoosterHandle handle, const void* indptr, int indptr_type,
                                                const int32_t* indices, const void* data, int data_type,
                                                int64_t nindptr, int64_t nelem, int64_t num_col, int predict_type,
                                                int start_iteration, int num_iteration, const char* parameter,
                                                int64_t* out_len, double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForCSRSingleRow(BoosterHandle handle, const void* indptr, int indptr_type,
                                                         const int32_t* indices, const void* data, int data_type,
                                                         int64_t nindptr, int64_t nelem, int64_t num_col,
                                                         int predict_type, int start_iteration, int num_iteration,
                                                         const char* parameter, int64_t* out_len, double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForCSC(BoosterHandle handle, const void* col_ptr, int col_ptr_type,
                                                const int32_t* indices, const void* data, int data_type,
                                                int64_t ncol_ptr, int64_t nelem, int64_t num_row, int predict_type,
                                                int start_iteration, int num_iteration, const char* parameter,
                                                int64_t* out_len, double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForMat(BoosterHandle handle, const void* data, int data_type, int32_t nrow,
                                                int32_t ncol, int is_row_major, int predict_type, int start_iteration,
                                                int num_iteration, const char* parameter, int64_t* out_len,
                                                double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForMatSingleRow(BoosterHandle handle, const void* data, int data_type,
                                                         int ncol, int is_row_major, int predict_type,
                                                         int start_iteration, int num_iteration,
                                                         const char* parameter, int64_t* out_len, double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForMats(BoosterHandle handle, const void** data, int data_type, int32_t nrow,
                                                 int32_t ncol, int predict_type, int start_iteration,
                                                 int num_iteration, const char* parameter, int64_t* out_len,
                                                 double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterSaveModel(BoosterHandle handle, int start_iteration, int num_iteration,
                                            int feature_importance_type, const char* filename);
LIGHTGBM_C_EXPORT int LGBM_BoosterSaveModelToString(BoosterHandle handle, int start_iteration, int num_iteration,
                                                    int feature_importance_type, int64_t buffer_len, int64_t* out_len,
                                                    char* out_str);
LIGHTGBM_C_EXPORT int LGBM_BoosterDumpModel(BoosterHandle handle, int start_iteration, int num_iteration,
                                            int feature_importance_type, int64_t buffer_len, int64_t* out_len,
                                            char* out_str);
LIGHTGBM_C_EXPORT int LGBM_BoosterConvertModelToIfElse(BoosterHandle handle, int num_iteration, int64_t buffer_len,
                                                       int64_t* out_len, char* out_str);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetLeafValue(BoosterHandle handle, int tree_idx, int leaf_idx, double* out_val);
LIGHTGBM_C_EXPORT int LGBM_BoosterSetLeafValue(BoosterHandle handle, int tree_idx, int leaf_idx, double val);
LIGHTGBM_C_EXPORT int LGBM_BoosterFeatureImportance(BoosterHandle handle, int num_iteration, int importance_type,
                                                    double* out_results);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetUpperBoundValue(BoosterHandle handle, double* out_results);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetLowerBoundValue(BoosterHandle handle, double* out_results);
LIGHTGBM_C_EXPORT int LGBM_BoosterGetDeviceName(BoosterHandle handle, int64_t buffer_len, int64_t* out_len,
                                                char* out_str);

/* ---- Network */
LIGHTGBM_C_EXPORT int LGBM_NetworkInit(const char* machines, int local_listen_port, int listen_time_out,
                                       int num_machines);
LIGHTGBM_C_EXPORT int LGBM_NetworkFree();
LIGHTGBM_C_EXPORT int LGBM_NetworkInitWithFunctions(int num_machines, int rank, void* reduce_scatter_ext_fun,
                                                    void* allgather_ext_fun);
LIGHTGBM_C_EXPORT int LGBM_SetMaxThreads(int num_threads);
LIGHTGBM_C_EXPORT int LGBM_GetMaxThreads(int* out);
LIGHTGBM_C_EXPORT int LGBM_GetEffectiveThreads(int* out);

/* ---- Arrow C data interface (struct ArrowArray / ArrowSchema, see lgap/arrow.h) */
struct ArrowArray;
struct ArrowSchema;
typedef void* ByteBufferHandle;
#define C_API_MATRIX_TYPE_CSR (0)
#define C_API_MATRIX_TYPE_CSC (1)
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromArrow(int64_t n_chunks, const struct ArrowArray* chunks,
                                                  const struct ArrowSchema* schema, const char* parameters,
                                                  const DatasetHandle reference, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetSetFieldFromArrow(DatasetHandle handle, const char* field_name, int64_t n_chunks,
                                                    const struct ArrowArray* chunks, const struct ArrowSchema* schema);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForArrow(BoosterHandle handle, int64_t n_chunks,
                                                  const struct ArrowArray* chunks, const struct ArrowSchema* schema,
                                                  int predict_type, int start_iteration, int num_iteration,
                                                  const char* parameter, int64_t* out_len, double* out_result);

/* ---- more dataset constructors */
// get_row_funptr: std::function<void(int idx, std::vector<std::pair<int, double>>& row)>*
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromCSRFunc(void* get_row_funptr, int num_rows, int64_t num_col,
                                                    const char* parameters, const DatasetHandle reference,
                                                    DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromSampledColumn(double** sample_data, int** sample_indices, int32_t ncol,
                                                          const int* num_per_col, int32_t num_sample_row,
                                                          int32_t num_local_row, int64_t num_dist_row,
                                                          const char* parameters, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_DatasetPushRowsByCSRWithMetadata(DatasetHandle dataset, const void* indptr,
                                                            int indptr_type, const int32_t* indices, const void* data,
                                                            int data_type, int64_t nindptr, int64_t nelem,
                                                            int64_t start_row, const float* label, const float* weight,
                                                            const double* init_score, const int32_t* query,
                                                            int32_t tid);
LIGHTGBM_C_EXPORT int LGBM_DatasetSerializeReferenceToBinary(DatasetHandle handle, ByteBufferHandle* out,
                                                             int32_t* out_len);
LIGHTGBM_C_EXPORT int LGBM_DatasetCreateFromSerializedReference(const void* ref_buffer, int32_t ref_buffer_size,
                                                                int64_t num_row, int32_t num_classes,
                                                                const char* parameters, DatasetHandle* out);
LIGHTGBM_C_EXPORT int LGBM_ByteBufferGetAt(ByteBufferHandle handle, int32_t index, uint8_t* out_val);
LIGHTGBM_C_EXPORT int LGBM_ByteBufferFree(ByteBufferHandle handle);

/* ---- single-row fast prediction (config parsed once) */
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForMatSingleRowFastInit(BoosterHandle handle, const int predict_type,
                                                                 const int start_iteration, const int num_iteration,
                                                                 const int data_type, const int32_t ncol,
                                                                 const char* parameter,
                                                                 FastConfigHandle* out_fastConfig);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForMatSingleRowFast(FastConfigHandle fastConfig_handle, const void* data,
                                                             int64_t* out_len, double* out_result);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForCSRSingleRowFastInit(BoosterHandle handle, const int predict_type,
                                                                 const int start_iteration, const int num_iteration,
                                                                 const int data_type, const int64_t num_col,
                                                                 const char* parameter,
                                                                 FastConfigHandle* out_fastConfig);
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictForCSRSingleRowFast(FastConfigHandle fastConfig_handle, const void* indptr,
                                                             const int indptr_type, const int32_t* indices,
                                                             const void* data, const int64_t nindptr,
                                                             const int64_t nelem, int64_t* out_len,
                                                             double* out_result);
LIGHTGBM_C_EXPORT int LGBM_FastConfigFree(FastConfigHandle fastConfig);

/* ---- sparse SHAP output */
LIGHTGBM_C_EXPORT int LGBM_BoosterPredictSparseOutput(BoosterHandle handle, const void* indptr, int indptr_type,
                                                      const int32_t* indices, const void* data, int data_type,
                                                      int64_t nindptr, int64_t nelem, int64_t num_col_or_row,
                                                      int predict_type, int start_iteration, int num_iteration,
                                                      const char* parameter, int matrix_type, int64_t* out_len,
                                                      void** out_indptr, int32_t** out_indices, void** out_data);
LIGHTGBM_C_EXPORT int LGBM_BoosterFreePredictSparse(void* indptr, int32_t* indices, void* data, int indptr_type,
                                                    int data_type);
LIGHTGBM_C_EXPORT void LGBM_SetLastError(const char* msg);

/* ---- MI355X device helpers (LambdaGap extension) */
LIGHTGBM_C_EXPORT int LGBM_DeviceCount(int* out);
// Waits for all queued device work of this process (timing brackets).
LIGHTGBM_C_EXPORT int LGBM_DeviceSynchronize();
// ---- kernel-level entry points (numerics tests / ops module)
// Gradients and hessians of the last boosting round (class-major); pass null buffers to query *out_len.
LIGHTGBM_C_EXPORT int LGBM_BoosterGetGradients(BoosterHandle handle, int64_t* out_len, float* grad, float* hess);
// Packed group layout: groups, total histogram bins, bytes per group bin, per-group histogram start.
LIGHTGBM_C_EXPORT int LGBM_DatasetGetGroupLayout(DatasetHandle handle, int* num_groups, int* num_total_bin,
                                                 int* bin_width, int32_t* hist_start);
// Row-major [num_data x num_groups] group bins.
LIGHTGBM_C_EXPORT int LGBM_DatasetGetGroupBins(DatasetHandle handle, uint16_t* out);
// (grad, hess) histogram over `rows` (null = all rows) built by the HIP histogram kernel:
// out_hist has 2 * num_total_bin doubles; group bin 0 (all features at their most frequent bin) stays 0.
LIGHTGBM_C_EXPORT int LGBM_DeviceHistogram(DatasetHandle handle, const float* grad, const float* hess,
                                           const int32_t* rows, int32_t num_rows, double* out_hist);
// Direct tests of the frontier engine's production kernels with a device learner configured by
// `parameters`: k_f_hist over k row subsets (rows concatenated, offsets[k + 1]) -> out
// [k][num_total_bin][2] at the kernel's fixed-point scale (quantized: integer level sums, levels
// [num_data] = g level << 8 | h level); k_f_partition of k parents -> the device's children lists
// and left counts next to the host learner's stable partition (exp_*).
LIGHTGBM_C_EXPORT int LGBM_DeviceTestFrontierHist(DatasetHandle handle, const char* parameters, const float* grad,
                                                  const float* hess, const int32_t* rows, const int32_t* offsets,
                                                  int k, double* out, uint16_t* levels);
// k_f_scan of the root round (all rows) next to the host split_math.h scan of the same histogram:
// out / ref [num_features][8] (gain, threshold, left count, default_left, left sum g, left sum h,
// valid, categorical thresholds).
LIGHTGBM_C_EXPORT int LGBM_DeviceTestFrontierScan(DatasetHandle handle, const char* parameters, const float* grad,
                                                  const float* hess, double* out, double* ref);
LIGHTGBM_C_EXPORT int LGBM_DeviceTestFrontierPartition(DatasetHandle handle, const char* parameters,
                                                       const int32_t* rows, const int32_t* offsets, int k,
                                                       const int32_t* feats, const int32_t* thr, const int32_t* dleft,
                                                       const uint32_t* catbits, int32_t* out_rows, int32_t* out_left,
                                                       int32_t* exp_rows, int32_t* exp_left);
// One device row-sampling pass (the HIP bagging / GOSS kernels) over host arrays: mode 1 bagging,
// 2 balanced bagging, 3 GOSS; `rounds` > 1 re-bags with the advanced streams and reports the last.
// grad/hess (num_class * num_rows, class-major) are scaled in place by GOSS. Returns the kept
// rows (ascending) in out_rows and their count in out_count.
LIGHTGBM_C_EXPORT int LGBM_DeviceSampleRows(int mode, int32_t num_rows, int num_class, float* grad, float* hess,
                                            const float* label, double fraction, double pos_fraction,
                                            double neg_fraction, double top_rate, double other_rate,
                                            int bagging_seed, uint32_t goss_seed, int rounds, int32_t* out_rows,
                                            int32_t* out_count);
LIGHTGBM_C_EXPORT int LGBM_DeviceCommGetUniqueId(char* out, int64_t buffer_len, int64_t* out_len);
LIGHTGBM_C_EXPORT int LGBM_DeviceCommInit(const char* unique_id, int64_t id_len, int num_ranks, int rank,
                                          int device_id);
LIGHTGBM_C_EXPORT int LGBM_DeviceCommFree();
LIGHTGBM_C_EXPORT int LGBM_PhaseTimerReport(int64_t buffer_len, int64_t* out_len, char* out_str);

#endif /* LGAP_C_API_H_ */
