# Package configuration for projects built outside the framework
# (reference contrib/build_with_parsec/CMakeLists.txt.in + PaRSECConfig.cmake):
#
#   find_package(ParsecAmd CONFIG REQUIRED PATHS <repo>/cmake)
#   add_executable(app main.cpp)
#   parsec_amd_add_jdf(app app.jdf)        # JDF -> C++ via parsec-ptgpp
#   target_link_libraries(app PRIVATE ParsecAmd::parsec)
#
# Generated sources of a JDF with BODY [type=HIP] are compiled as HIP for
# gfx950 (CMAKE_HIP_ARCHITECTURES); the project must enable_language(HIP).
get_filename_component(PARSEC_AMD_ROOT "${CMAKE_CURRENT_LIST_DIR}/.." ABSOLUTE)
set(PARSEC_AMD_PTGPP "${PARSEC_AMD_ROOT}/parsec_amd/bin/parsec-ptgpp")
set(PARSEC_AMD_LIBRARY "${PARSEC_AMD_ROOT}/parsec_amd/lib/libparsec_amd.so")
if(NOT EXISTS "${PARSEC_AMD_LIBRARY}" OR NOT EXISTS "${PARSEC_AMD_PTGPP}")
  set(ParsecAmd_FOUND FALSE)
  set(ParsecAmd_NOT_FOUND_MESSAGE "framework not built: run python -m parsec_amd._build in ${PARSEC_AMD_ROOT}")
  return()
endif()
if(NOT DEFINED ROCM_PATH)
  set(ROCM_PATH "/opt/rocm")
endif()

if(NOT TARGET ParsecAmd::parsec)
  add_library(ParsecAmd::parsec SHARED IMPORTED)
  set_target_properties(ParsecAmd::parsec PROPERTIES
    IMPORTED_LOCATION "${PARSEC_AMD_LIBRARY}"
    INTERFACE_INCLUDE_DIRECTORIES "${PARSEC_AMD_ROOT}/include;${PARSEC_AMD_ROOT}/csrc;${ROCM_PATH}/include"
    INTERFACE_COMPILE_DEFINITIONS "__HIP_PLATFORM_AMD__"
    INTERFACE_COMPILE_FEATURES "cxx_std_20"
    INTERFACE_LINK_LIBRARIES "${ROCM_PATH}/lib/libamdhip64.so;pthread")
endif()

include("${CMAKE_CURRENT_LIST_DIR}/ParsecAmdPTG.cmake")
set(ParsecAmd_FOUND TRUE)
