// SiftGPU.h -- C++ API of the MI355X SIFT library (libsiftgpu.so), drop-in for the reference's
// SiftGPU/SiftGPU.h.
//
// Binary compatibility contract (reference SiftGPU/SiftGPU.h): callers such as
// TestWin/SimpleSIFT.cpp dlopen the library, resolve the extern "C" factories and then call
// VIRTUAL methods through this class layout, and read the public data members _timing and
// _imgpath.  Therefore:
//   * the data members of SiftParam / SiftGPU / SiftMatchGPU have the reference's types, order
//     and sizes (SiftGPU.h:57-86, 110-139, 267-270), so offsets match; private state the MI355X
//     runtime needs hangs off the reference's pointer slots;
//   * the virtual functions are declared in the reference's order (SiftGPU.h:142-196,
//     271-334), so the Itanium vtables match slot for slot;
//   * the factories are extern "C" (SiftGPU.h:49, 344-359).
// Everything behind these declarations is new: the work runs on gfx950 HIP kernels through the
// C ABI of include/sgpu.h.  GL enumerants are accepted by value (GL_LUMINANCE 0x1909, GL_RGB
// 0x1907, GL_RGBA 0x1908, GL_BGR 0x80E0, GL_BGRA 0x80E1, GL_LUMINANCE_ALPHA 0x190A;
// GL_UNSIGNED_BYTE 0x1401, GL_UNSIGNED_SHORT 0x1403, GL_FLOAT 0x1406); no OpenGL is needed.
#ifndef GPU_SIFT_H
#define GPU_SIFT_H

#include <stddef.h>

#define SIFTGPU_EXPORT __attribute__((visibility("default")))
#define SIFTGPU_EXPORT_EXTERN extern "C" __attribute__((visibility("default")))

class SiftParam {
public:
    float* _sigma;            // filter sigma per level step
    float _sigma_skip0;
    float _sigma_skip1;
    float _sigma0;            // sigma of the first level
    float _sigman;
    int _sigma_num;
    int _dog_level_num;       // DoG levels per octave
    int _level_num;
    int _level_min;
    int _level_max;
    int _level_ds;
    float _dog_threshold;
    float _edge_threshold;
    void ParseSiftParam();
public:
    float GetLevelSigma(int lev);
    float GetInitialSmoothSigma(int octave_min);
    SIFTGPU_EXPORT SiftParam();
};

class LiteWindow;
class GLTexInput;
class ShaderMan;
class SiftPyramid;
class ImageList;

class SiftGPU : public SiftParam {
public:
    enum { SIFTGPU_NOT_SUPPORTED = 0, SIFTGPU_PARTIAL_SUPPORTED = 1, SIFTGPU_FULL_SUPPORTED = 2 };
    typedef struct SiftKeypoint { float x, y, s, o; } SiftKeypoint;
protected:
    int _current;
    int _initialized;
    int _image_loaded;
    char* _imgpath;
    char* _outpath;
    ImageList* _list;
    GLTexInput* _texImage;     // MI355X: host-side input image holder
    SiftPyramid* _pyramid;     // MI355X: runtime state (device context, options, results)
    static void PrintUsage();
    void InitSiftGPU();
    void LoadImageList(const char* imlist);
public:
    float _timing[10];         // seconds: [0] load, [1] init, [2..] stage times
    inline const char* GetCurrentImagePath() { return _imgpath; }
public:
    SIFTGPU_EXPORT virtual void SetImageList(int nimage, const char** filelist);
    SIFTGPU_EXPORT virtual int GetFeatureNum();
    SIFTGPU_EXPORT virtual void SaveSIFT(const char* szFileName);
    SIFTGPU_EXPORT virtual void GetFeatureVector(SiftKeypoint* keys, float* descriptors);
    SIFTGPU_EXPORT virtual void SetKeypointList(int num, const SiftKeypoint* keys,
                                                int keys_have_orientation = 1);
    SIFTGPU_EXPORT virtual int CreateContextGL();
    SIFTGPU_EXPORT virtual int VerifyContextGL();
    SIFTGPU_EXPORT virtual int IsFullSupported();
    SIFTGPU_EXPORT virtual void SetVerbose(int verbose = 4);
    inline void SetVerboseBrief() { SetVerbose(2); }
    SIFTGPU_EXPORT virtual void ParseParam(int argc, char** argv);
    SIFTGPU_EXPORT virtual int RunSIFT(const char* imgpath);
    SIFTGPU_EXPORT virtual int RunSIFT(int index);
    SIFTGPU_EXPORT virtual int RunSIFT(int width, int height, const void* data,
                                       unsigned int gl_format, unsigned int gl_type);
    SIFTGPU_EXPORT virtual int RunSIFT();
    SIFTGPU_EXPORT virtual int RunSIFT(int num, const SiftKeypoint* keys,
                                       int keys_have_orientation = 1);
    SIFTGPU_EXPORT SiftGPU(int np = 1);
    SIFTGPU_EXPORT virtual ~SiftGPU();
    SIFTGPU_EXPORT virtual void SetActivePyramid(int index) {}
    SIFTGPU_EXPORT virtual int GetImageCount();
    SIFTGPU_EXPORT virtual void SetTightPyramid(int tight = 1);
    SIFTGPU_EXPORT virtual int AllocatePyramid(int width, int height);
    SIFTGPU_EXPORT virtual void SetMaxDimension(int sz);
public:
    SIFTGPU_EXPORT void* operator new(size_t size);
};

class SiftMatchGPU {
public:
    enum SIFTMATCH_LANGUAGE {
        SIFTMATCH_SAME_AS_SIFTGPU = 0,
        SIFTMATCH_GLSL = 2,
        SIFTMATCH_CUDA = 3,         // MI355X: "GPU device 0"; +i selects device i
        SIFTMATCH_CUDA_DEVICE0 = 3
    };
private:
    int __max_sift;
    int __language;
    SiftMatchGPU* __matcher;        // MI355X: runtime state
    virtual void InitSiftMatch() {}
protected:
    SIFTGPU_EXPORT virtual int _CreateContextGL();
    SIFTGPU_EXPORT virtual int _VerifyContextGL();
public:
    inline int CreateContextGL() { return _CreateContextGL(); }
    inline int VerifyContextGL() { return _VerifyContextGL(); }
    SIFTGPU_EXPORT SiftMatchGPU(int max_sift = 14096);
    SIFTGPU_EXPORT virtual void SetLanguage(int gpu_language);
    SIFTGPU_EXPORT virtual void SetDeviceParam(int argc, char** argv);
    SIFTGPU_EXPORT virtual void SetMaxSift(int max_sift);
    SIFTGPU_EXPORT virtual ~SiftMatchGPU();
    SIFTGPU_EXPORT virtual void SetDescriptors(int index, int num, const float* descriptors,
                                               int id = -1);
    SIFTGPU_EXPORT virtual void SetDescriptors(int index, int num,
                                               const unsigned char* descriptors, int id = -1);
    SIFTGPU_EXPORT virtual int GetSiftMatch(int max_match, int match_buffer[][2],
                                            float distmax = 0.7, float ratiomax = 0.8,
                                            int mutual_best_match = 1);
    SIFTGPU_EXPORT virtual void SetFeautreLocation(int index, const float* locations,
                                                   int gap = 0);
    inline void SetFeatureLocation(int index, const SiftGPU::SiftKeypoint* keys) {
        SetFeautreLocation(index, (const float*)keys, 2);
    }
    SIFTGPU_EXPORT virtual int GetGuidedSiftMatch(int max_match, int match_buffer[][2],
                                                  float H[3][3], float F[3][3],
                                                  float distmax = 0.7, float ratiomax = 0.8,
                                                  float hdistmax = 32, float fdistmax = 16,
                                                  int mutual_best_match = 1);
public:
    SIFTGPU_EXPORT void* operator new(size_t size);
};

typedef SiftGPU::SiftKeypoint SiftKeypoint;

SIFTGPU_EXPORT_EXTERN SiftGPU* CreateNewSiftGPU(int np = 1);
SIFTGPU_EXPORT_EXTERN SiftMatchGPU* CreateNewSiftMatchGPU(int max_sift = 14096);

class ComboSiftGPU : public SiftGPU, public SiftMatchGPU {
public:
    SIFTGPU_EXPORT void* operator new(size_t size);
};
SIFTGPU_EXPORT_EXTERN ComboSiftGPU* CreateComboSiftGPU();
// No TCP server on this platform: returns a local ComboSiftGPU (multi-GPU is in-process).
SIFTGPU_EXPORT_EXTERN ComboSiftGPU* CreateRemoteSiftGPU(int port = 7777,
                                                        char* remote_server = NULL);

SIFTGPU_EXPORT int CreateLiteWindow(LiteWindow* window);
SIFTGPU_EXPORT void RunServerLoop(int port, int argc, char** argv);

#endif  // GPU_SIFT_H
