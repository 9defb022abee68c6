/*
 * hs_types.h — plain-C data contract of the photometric-BA hot path.
 *
 * These PODs are what crosses the drop-in boundary (include/hs_ba.h,
 * include/hs_track.h, include/hs_trace.h).  They re-express the reference's
 * shared_ptr object graph (FrameShell -> Frame -> MapPoint ->
 * PointFrameResidual) as flat structure-of-arrays that the
 * caller owns; the library copies them in.  No torch / Eigen / HIP types.
 *
 * Reference types replaced:
 *   hs_camera   <- CalibData value_scaled + pyramid rule   (Include/CalibData.h:60-193)
 *   hs_frame    <- FrameOptimizationData state/evalPT       (Include/Frame.h:116-275)
 *   hs_points   <- MapPoint + MapPointOptimizationData      (Include/MapPoint.h:16-115)
 *   hs_residuals<- PointFrameResidual (host/target/state)   (Include/OptimizationClasses.h:79-163)
 *   hs_params   <- the setting_* globals read on the path   (Src/Settings.cpp)
 */
#ifndef HS_TYPES_H
#define HS_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HS_PATTERN_NUM 8   /* staticPattern[8], Include/GlobalTypes.h:181-184,225-228 */
#define HS_CPARS 4         /* Include/GlobalTypes.h:223 */
#define HS_MAX_FRAMES 8    /* 7 KF + 1 transient during optimize (SURVEY.md §0 note a) */
#define HS_MAX_LEVELS 6    /* DirPyrLevels upper bound (Src/Settings.cpp:28) */

/* ResState, Include/GlobalTypes.h:85 */
enum { HS_RES_IN = 0, HS_RES_OOB = 1, HS_RES_OUT = 2 };

/* status codes returned by every entry point */
enum {
  HS_OK = 0,
  HS_ERR_INVALID = -1,     /* bad argument / shape */
  HS_ERR_HIP = -2,         /* HIP runtime failure */
  HS_ERR_RCCL = -3,        /* collective failure */
  HS_ERR_NONFINITE = -4,   /* NaN/Inf energy or system (reference: isLost) */
  HS_ERR_STATE = -5,       /* call order violated (e.g. no window set) */
  HS_ERR_NOMEM = -6
};

typedef struct hs_camera {
  int width, height;   /* level-0 size (CalibData::Width/Height) */
  int n_levels;        /* direct pyramid levels (CalibData ctor rule, Include/CalibData.h:107-130) */
  int pad;
  float fx, fy, cx, cy;/* CalibData::value_scaledf at level 0 */
} hs_camera;

typedef struct hs_frame {
  double worldToCam_evalPT[7]; /* Sophus SE3d::data(): qx qy qz qw tx ty tz */
  double state[10];            /* FrameOptimizationData::state (unscaled, Include/Frame.h:129) */
  double state_zero[10];       /* FrameOptimizationData::state_zero */
  float ab_exposure;           /* FrameShell::ab_exposure */
  float frameEnergyTH;         /* Frame::frameEnergyTH (Src/Frame.cpp:47 default 8*8*8) */
  int id;                      /* FrameOptimizationData::id; id==0 gets the strong pose prior (Include/Frame.h:230-258) */
  int pad;
} hs_frame;

typedef struct hs_points {
  int n;                       /* number of active points; MUST be sorted by host */
  const int* host;             /* [n] host frame index in the window */
  const float* u;              /* [n] */
  const float* v;              /* [n] */
  const float* idepth;         /* [n] MapPoint::idepth */
  const float* idepth_zero;    /* [n] MapPointOptimizationData::idepth_zero */
  const float* color;          /* [n*8] MapPoint::color */
  const float* weights;        /* [n*8] MapPoint::weights */
  const uint8_t* has_depth_prior; /* [n] nullable (=> false) */
} hs_points;

typedef struct hs_residuals {
  int n;                       /* MUST be grouped by point, points in hs_points order */
  const int* point;            /* [n] */
  const int* target;           /* [n] target frame index */
  const uint8_t* state;        /* [n] initial ResState, nullable (=> IN, as resetOOB) */
} hs_residuals;

/* Hot-path settings (Src/Settings.cpp).  hs_params_default() fills these. */
typedef struct hs_params {
  float huberTH;                 /* 9      :68 */
  float outlierTHSumComponent;   /* 2500   :64 */
  float frameEnergyTHN;          /* 0.7    :73 */
  float frameEnergyTHFacMedian;  /* 1.5    :74 */
  float frameEnergyTHConstWeight;/* 0.5    :75 */
  float overallEnergyTHWeight;   /* 1      :66 */
  float idepthFixPrior;          /* 2500   :100 */
  float initialCalibHessian;     /* 5e9    :106 */
  float affineOptModeA;          /* 1e12   :109 */
  float affineOptModeB;          /* 1e8    :110 */
  float initialRotPrior;         /* 1e11   :102 */
  float initialTransPrior;       /* 1e10   :103 */
  float initialAffAPrior;        /* 1e14   :105 */
  float initialAffBPrior;        /* 1e14   :104 */
  double solverModeDelta;        /* 1e-5   :115 */
  float thOptIterations;         /* 1.2    :62 */
  float coarseCutoffTH;          /* 20     :77 */
  int minOptIterations;          /* 1      :61 */
  int pad;
  /* ImmaturePoint (ctor + traceOn, Src/ImmaturePoint.cpp:7-350) */
  float outlierTH;               /* 12*12  :65 */
  float maxPixSearch;            /* 0.027  :85 */
  float trace_slackInterval;     /* 1.5    :87 */
  float trace_stepsize;          /* 1      :88 */
  float trace_minImprovementFactor; /* 2   :89 */
  float trace_GNThreshold;       /* 0.1    :92 */
  float trace_extraSlackOnTH;    /* 1.2    :93 */
  int minTraceTestRadius;        /* 2      :90 */
  int trace_GNIterations;        /* 3      :91 */
  /* marginalization (EnergyFunctional::marginalizePointsF, Src/EnergyFunctional.cpp:563,601) */
  float idepthFixPriorMargFac;   /* 600*600 :101 */
  float margWeightFac;           /* 0.25   :80 */
  /* point activation (System::activatePointsMT + optimizeImmaturePoint, Src/Mapping.cpp:330-492,
     Src/FullSystemOptPoint.cpp:24-175) */
  float desiredPointDensity;     /* 2000   :121 */
  float minTraceQuality;         /* 3      :86 */
  float minIdepthH_act;          /* 100    :118 */
  int GNItsOnPointActivation;    /* 3      :54 */
  /* PixelSelector (Src/PixelSelector.cpp:54-418) */
  float minGradHistCut;          /* 0.5    :29 */
  float minGradHistAdd;          /* 7      :30 */
  float gradDownweightPerLevel;  /* 0.75   :31 */
  int selectDirectionDistribution; /* 1    :32 */
} hs_params;

#ifdef __cplusplus
}
#endif
#endif /* HS_TYPES_H */
