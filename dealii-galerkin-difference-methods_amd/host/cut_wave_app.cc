// cut_wave_app -- applications/wave/wave-app.cc over the C ABI: the wave
// application's presets (step85, heat / heat-rk / heat-impl, heat-composite,
// wave, wave-composite; dim 1 and 2 as the reference's tests run them) through
// GDM::HIP::CutWave::WaveProblem (gdm/hip/cut_wave.h), printing the
// reference's postprocess lines ("%5d %8.5f %14.8e %14.8e %14.8e").
//
//   cut_wave_app DIM SIMULATION [DEVICE]
#include <gdm/hip/cut_wave.h>

#include <cstdio>
#include <cstdlib>
#include <string>

using namespace GDM::HIP::CutWave;

template <int dim>
static void run(const std::string &name, int device) {
  Parameters<dim> params;
  fill_parameters(params, name);
  WaveProblem<dim>(params, device).run();
}

int main(int argc, char **argv) {
  if (argc < 3 || std::string(argv[1]) == "--help") {
    std::printf("Usage: ./cut_wave_app dim simulation [device]\n\n");
    std::printf("dim         number of dimensions (1-2)\n");
    std::printf("simulation  name of simulation (step85, heat, heat-rk, heat-impl, heat-composite, wave, wave-composite)\n");
    return argc < 3 ? 1 : 0;
  }
  const int dim = std::atoi(argv[1]);
  const std::string name = argv[2];
  const int device = argc > 3 ? std::atoi(argv[3]) : 0;
  try {
    if (dim == 1)
      run<1>(name, device);
    else if (dim == 2)
      run<2>(name, device);
    else
      throw GDM::HIP::Error("dim must be 1 or 2");
  } catch (const std::exception &e) {
    std::fprintf(stderr, "cut_wave_app: %s\n", e.what());
    return 1;
  }
  return 0;
}
