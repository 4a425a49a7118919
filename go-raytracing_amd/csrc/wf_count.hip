// wf_count.hip — one variant group of the wavefront pipeline (ring 8, instrumented (work-counting) kernels),
// instantiated in its own translation unit so the groups compile in parallel
// (wavefront.hip, RTG_WF_GROUP).
#define RTG_WF_GROUP 2
#include "wavefront.hip"
