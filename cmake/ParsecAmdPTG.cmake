# parsec_amd_add_jdf(<target> <file.jdf> [<file.jdf> ...])
# Runs parsec-ptgpp on each .jdf and adds the generated C++ (and header
# directory) to <target>. A JDF with a BODY [type=HIP] is compiled as HIP.
# Mirrors the reference's target_ptg_sources
# (cmake_modules/ParsecCompilePTG.cmake:142-150).
function(parsec_amd_add_jdf target)
  if(DEFINED PARSEC_AMD_PTGPP)
    set(ptgpp ${PARSEC_AMD_PTGPP})
  else()
    set(ptgpp parsec-ptgpp)  # in-tree target
  endif()
  foreach(jdf ${ARGN})
    get_filename_component(jdf ${jdf} ABSOLUTE)
    get_filename_component(name ${jdf} NAME_WE)
    set(out ${CMAKE_CURRENT_BINARY_DIR}/${name})
    add_custom_command(
      OUTPUT ${out}.cpp ${out}.h
      COMMAND ${ptgpp} -i ${jdf} -o ${out} -f ${name}
      DEPENDS ${jdf}
      COMMENT "parsec-ptgpp ${name}.jdf")
    file(READ ${jdf} src)
    string(REPLACE " " "" src "${src}")
    if(src MATCHES "type=HIP")
      set_source_files_properties(${out}.cpp PROPERTIES LANGUAGE HIP)
    endif()
    target_sources(${target} PRIVATE ${out}.cpp)
    target_include_directories(${target} PRIVATE ${CMAKE_CURRENT_BINARY_DIR})
  endforeach()
endfunction()
