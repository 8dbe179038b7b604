# parsec_amd_add_jdf(<target> <file.jdf> [<file.jdf> ...])
# Runs parsec-ptgpp on each .jdf and adds the generated C++ (and header
# directory) to <target>. Mirrors the reference's target_ptg_sources
# (cmake_modules/ParsecCompilePTG.cmake:142-150).
function(parsec_amd_add_jdf target)
  foreach(jdf ${ARGN})
    get_filename_component(name ${jdf} NAME_WE)
    set(out ${CMAKE_CURRENT_BINARY_DIR}/${name})
    add_custom_command(
      OUTPUT ${out}.cpp ${out}.h
      COMMAND parsec-ptgpp -i ${jdf} -o ${out} -f ${name}
      DEPENDS ${jdf} parsec-ptgpp
      COMMENT "parsec-ptgpp ${name}.jdf")
    target_sources(${target} PRIVATE ${out}.cpp)
    target_include_directories(${target} PRIVATE ${CMAKE_CURRENT_BINARY_DIR})
  endforeach()
endfunction()
