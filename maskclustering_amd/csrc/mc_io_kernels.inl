// mc_io_kernels.inl — frame decode on the device (the step before S1).
//
// dataset/scannet.py:49-54 (and matterport.py:92, scannetpp.py:169): depth = uint16 / depth_scale
// in float64, stored as float32.  dataset/scannet.py:68-73: the segmentation resized to the depth
// size with cv2.INTER_NEAREST; the source row / column of every output row / column comes in as
// two index tables (OpenCV's resizeNN tables, built on the host), so one thread per output pixel
// does one gather.  Frames are independent: the launch covers F x H x W pixels.

namespace mc {

__global__ __launch_bounds__(256) void k_frames_decode(int64_t total, int Hd, int Wd, int Hs, int Ws,
                                                       const unsigned short *__restrict__ depth_in, double scale,
                                                       const unsigned char *__restrict__ seg_in,
                                                       const int *__restrict__ y_ofs, const int *__restrict__ x_ofs,
                                                       float *__restrict__ depth_out, unsigned char *__restrict__ seg_out)
{
    const int64_t plane = static_cast<int64_t>(Hd) * Wd;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
        const int64_t f = i / plane, r = i % plane;
        const int y = static_cast<int>(r / Wd), x = static_cast<int>(r % Wd);
        if (depth_in) depth_out[i] = static_cast<float>(static_cast<double>(depth_in[i]) / scale);
        if (seg_in) seg_out[i] = seg_in[f * static_cast<int64_t>(Hs) * Ws + static_cast<int64_t>(y_ofs[y]) * Ws + x_ofs[x]];
    }
}

}  // namespace mc
