// Graphics.h — the reference's static render-backend class (Graphics.h:117-134), re-implemented
// over the rmr C ABI (include/rmr.h). Host code written against the reference's Graphics compiles
// against this header with two differences, both forced by the missing dependencies:
//   * addMaterial / addObject take the JSON text of one material / object (the reference takes a
//     jsoncpp Json::Value, which is not part of this toolchain);
//   * Display() (the GL preview, Graphics.cpp:356-390) is not provided: there is no window.
// Error behaviour follows the reference: every member is void and failures are printed to stderr;
// lastStatus() / lastError() expose the rmr status for callers that want to check.
#pragma once
#include <string>
#include <vector>

#include "../../include/rmr.h"
#include "../../include/rmr_group.h"
#include "Vector.h"

class Graphics {
public:
    // Graphics::Init (Graphics.cpp:263-312): create the device context and the accumulator.
    static void Init();
    // Graphics::Render (Graphics.cpp:314-354): ONE sample for every pixel with min <= pix < max,
    // running mean with index currentSample (0 overwrites).
    static void Render(float currentTime, Vector::Vector2 min, Vector::Vector2 max, unsigned currentSample);
    // Batched form of `nspp` consecutive Render calls over the integer rect (bitwise equal).
    static void RenderSamples(const float* times, Vector::Vector2 min, Vector::Vector2 max,
                              unsigned firstSample, unsigned nspp);
    // Graphics::Reload (Graphics.cpp:392-752): compile the scene, apply the image size, clear.
    static void Reload();
    // Graphics::SaveImage (Graphics.cpp:754-799): 24-bit BMP with the reference's encoding.
    static void SaveImage(std::string path);
    // Graphics::addMaterial / addObject / clearScene (Graphics.cpp:801-815): store by value.
    static void addMaterial(const std::string& materialJson);
    static void addObject(const std::string& objectJson);
    static void clearScene();
    // Graphics::setImageSize / getImageSize (Graphics.cpp:817-825): applied at the next Reload.
    static void setImageSize(Vector::Vector2 size);
    static Vector::Vector2 getImageSize();
    // Graphics::setView (Graphics.cpp:827-835): the 3rd argument feeds uniform "ray01", the 4th
    // "ray10" (Camera.cpp:101 passes its ray10 third).
    static void setView(Vector::Vector3 eye, Vector::Vector3 ray00, Vector::Vector3 ray01,
                        Vector::Vector3 ray10, Vector::Vector3 ray11);

    // ---- rmr extensions (not in the reference) -------------------------------------------------
    // Shader variant: RMR_VARIANT_RM1/RM2/RM3. The reference hard-wires RayMarch3 (Graphics.cpp:272).
    static void setVariant(int variant);
    static int getVariant();
    static void setParams(const rmr_params& p);
    static rmr_params getParams();
    static void setDevice(int device);
    // Several GPUs of the node from this process (librmr_group.so, include/rmr_group.h): call before
    // Init. Init then creates a device group instead of one context; setView / setParams / setEnvMap /
    // Reload go to every GPU, RenderFrame renders whole frames tile-partitioned over them with one RCCL
    // reduce each, and SaveImage writes the last such frame. (Render / RenderSamples draw on the first
    // GPU's context alone.) One device is a valid group: the RCCL path with a single rank.
    static void setDevices(const std::vector<int>& devices);
    // One whole frame of samples 0 .. nspp-1 (times[k] seeds sample k): on the device group when
    // setDevices was given, else rmr_render_spp of the whole image on the one context. Bitwise the
    // same image either way.
    static void RenderFrame(const float* times, unsigned nspp);
    static rmr_group* group();  // the device group (nullptr without setDevices)
    // envTex of skyColor (Graphics.cpp:287 loads it from data/textures/veranda_1k.hdr): RGBA8, row
    // 0 = up; used when the params' use_env_tex is set. nullptr removes it.
    static void setEnvMap(const unsigned char* rgba8, int w, int h);
    static void Sync();
    static bool saveCheckpoint(const std::string& path, unsigned samplesDone);
    static bool loadCheckpoint(const std::string& path, unsigned* samplesDone);
    static int lastStatus();
    static std::string lastError();
    static rmr_ctx* context();  // the underlying C-ABI context (nullptr before Init)
    static void Shutdown();
};
